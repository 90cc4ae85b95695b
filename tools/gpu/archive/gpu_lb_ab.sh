# Wide kernel occupancy A/B: __launch_bounds__ min blocks 2 (default) vs 4/5/6.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/lb_$n.json 2> gpurun_out/lb_$n.err || { tail -30 gpurun_out/lb_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/lb_$n.json'));r=d['roofline'];print('probe %.2f ms  frac %.3f'%(r['probe_ms_avg'],r['frac']))"
}
for v in "" lb4 lb5 lb6; do
  run mlst_$v "$v" --workload mlst
  run d1000_$v "$v" --docs 1000 --genome-len 1000000
  run d2000_$v "$v" --docs 2000 --genome-len 1000000
done
