# Where the wide kernel's time goes: counting skipped (measurement-only build) and hit matrix not written.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/nc_$n.json 2> gpurun_out/nc_$n.err || { tail -30 gpurun_out/nc_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/nc_$n.json'));r=d['roofline'];print('probe %.2f ms  frac %.3f'%(r['probe_ms_avg'],r['frac']))"
}
run mlst "" --workload mlst
run mlst_nocount nocount --workload mlst
run mlst_tot "" --workload mlst --totals-only
run mlst_nocount_tot nocount --workload mlst --totals-only
run d1000 "" --docs 1000 --genome-len 1000000
run d1000_nocount nocount --docs 1000 --genome-len 1000000
run d2000 "" --docs 2000 --genome-len 1000000
run d2000_nocount nocount --docs 2000 --genome-len 1000000
