set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/par.log 2>&1 || { tail -30 gpurun_out/par.log; exit 9; }
tail -1 gpurun_out/par.log
run() {  # name, args...
  n=$1; shift
  echo "== $n: $*"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/after_$n.json 2> gpurun_out/after_$n.err || { tail -30 gpurun_out/after_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/after_$n.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms probe %.2f ms  frac %.3f  bank %.2f GB'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac'],d['config']['bank_device_bytes']/1e9))"
}
run d1000 --docs 1000 --genome-len 1000000
XSPECT2_AMD_WIDE_P=2 run d1000p2 --docs 1000 --genome-len 1000000
run d600 --docs 600 --genome-len 1000000
run d300 --docs 300 --genome-len 1000000
run d2000 --docs 2000 --genome-len 1000000
run mlst --workload mlst
run species
