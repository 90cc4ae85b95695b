# Row compaction on compact banks (XS_WIDE_COMPACT_ROWS) A/B: parity of the default build, MLST bench both ways.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par_cr.log 2>&1 || { tail -40 gpurun_out/par_cr.log; exit 9; }
echo "parity: $(tail -1 gpurun_out/par_cr.log)"
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/cr_$n.json 2> gpurun_out/cr_$n.err || { tail -30 gpurun_out/cr_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/cr_$n.json'));r=d['roofline'];print('step %.2f ms  probe %.2f ms  frac %.3f'%(d['ms_per_step'],r['probe_ms_avg'],r['frac']))"
}
run mlst_cr "" --workload mlst
run mlst_off nocr --workload mlst
run mlst_cr2 "" --workload mlst
run mlst_off2 nocr --workload mlst
