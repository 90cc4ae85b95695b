# After splitting the probe families into translation units: GPU tests, then
# MLST / species A/B against the pre-session library (libxspect_hip.old.so).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -1 gpurun_out/gpu_tests.log
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { tail -30 gpurun_out/ab_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$n.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms probe %.2f ms  frac %.3f'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac']))"
}
run mlst_old1 old --workload mlst
run mlst_new1 "" --workload mlst
run mlst_old2 old --workload mlst
run mlst_new2 "" --workload mlst
run species_new "" 
run species_old old
