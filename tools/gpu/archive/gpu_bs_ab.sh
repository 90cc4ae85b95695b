# Bit-sliced row accumulation A/B (XS_WIDE_BITSLICE planes 2/3/4 vs off); parity of each variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in bs2 bs3 bs4; do
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "classic or compact" > gpurun_out/par_$v.log 2>&1 || { tail -30 gpurun_out/par_$v.log; exit 9; }
  echo "$v parity: $(tail -1 gpurun_out/par_$v.log)"
done
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/bs_$n.json 2> gpurun_out/bs_$n.err || { tail -30 gpurun_out/bs_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/bs_$n.json'));r=d['roofline'];print('probe %.2f ms  frac %.3f'%(r['probe_ms_avg'],r['frac']))"
}
for v in "" bs2 bs3 bs4; do
  run mlst_$v "$v" --workload mlst
  run d300_$v "$v" --docs 300 --genome-len 1000000
done
