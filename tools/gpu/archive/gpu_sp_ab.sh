# Sparse LDS counting on compact banks (XS_WIDE_SPARSE) A/B; parity of the variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
XSPECT2_AMD_LIB_VARIANT=sp timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par_sp.log 2>&1 || { tail -30 gpurun_out/par_sp.log; exit 9; }
echo "sp parity: $(tail -1 gpurun_out/par_sp.log)"
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/sp_$n.json 2> gpurun_out/sp_$n.err || { tail -30 gpurun_out/sp_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/sp_$n.json'));r=d['roofline'];print('probe %.2f ms  frac %.3f'%(r['probe_ms_avg'],r['frac']))"
}
run mlst_off "" --workload mlst
run mlst_sp sp --workload mlst
run mlst_off2 "" --workload mlst
run mlst_sp2 sp --workload mlst
