# Compact banks on the wide kernel (C lanes per k-mer per group): GPU parity,
# then MLST with 1/2/4 sub-tiles in flight against the slot kernel (old lib).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -1 gpurun_out/gpu_tests.log
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v] P=${XSPECT2_AMD_WIDEG_P:-2}: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/wg_$n.json 2> gpurun_out/wg_$n.err || { tail -30 gpurun_out/wg_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/wg_$n.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms probe %.2f ms  frac %.3f'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac']))"
}
XSPECT2_AMD_WIDEG_P=1 run mlst_p1 "" --workload mlst
XSPECT2_AMD_WIDEG_P=2 run mlst_p2 "" --workload mlst
XSPECT2_AMD_WIDEG_P=4 run mlst_p4 "" --workload mlst
run mlst_slots old --workload mlst
