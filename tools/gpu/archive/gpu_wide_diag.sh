# Where does a wide (D=1000) probe spend its time?  Bank size x hit-matrix write.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, args...
  n=$1; shift
  echo "== $n: $*"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/diag_$n.json 2> gpurun_out/diag_$n.err || { tail -30 gpurun_out/diag_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/diag_$n.json'));r=d['roofline'];print('value %.3e probes/s  probe %.2f ms  frac %.3f  bank %.2f GB'%(d['value'],r['probe_ms_avg'],r['frac'],d['config']['bank_device_bytes']/1e9))"
}
run d1000_hits --docs 1000 --genome-len 1000000
run d1000_tot --docs 1000 --genome-len 1000000 --totals-only
run d1000s_hits --docs 1000 --genome-len 200000
run d1000s_tot --docs 1000 --genome-len 200000 --totals-only
run d600_hits --docs 600 --genome-len 1000000
run d100_tot --docs 100 --totals-only
run d128_hits --docs 128 --genome-len 1000000
run d200_hits --docs 200 --genome-len 1000000
