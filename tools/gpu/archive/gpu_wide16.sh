# Wide kernel at 16 chunk lanes (D 1025..2048) and the loads-in-flight (P) sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 9; }
tail -1 gpurun_out/par.log
run() {  # name, args...
  n=$1; shift
  echo "== $n P=${XSPECT2_AMD_WIDE_P:-1}: $*"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/w16_$n.json 2> gpurun_out/w16_$n.err || { tail -30 gpurun_out/w16_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/w16_$n.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms probe %.2f ms  frac %.3f  bank %.2f GB'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac'],d['config']['bank_device_bytes']/1e9))"
}
for P in 1 2 4; do
  XSPECT2_AMD_WIDE_P=$P run d2000p$P --docs 2000 --genome-len 1000000
done
XSPECT2_AMD_WIDE_P=4 run d1000p4 --docs 1000 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d1000p2 --docs 1000 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d600p2 --docs 600 --genome-len 1000000
XSPECT2_AMD_WIDE_P=4 run d600p4 --docs 600 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d300p2 --docs 300 --genome-len 1000000
XSPECT2_AMD_WIDE_P=1 run d200p1 --docs 200 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d200p2 --docs 200 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d1500p2 --docs 1500 --genome-len 1000000
