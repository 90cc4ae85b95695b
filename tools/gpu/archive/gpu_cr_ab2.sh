# Row compaction A/B on WGS-like MLST input (reads from outside every locus).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, variant, args...
  n=$1; v=$2; shift 2
  echo "== $n [$v]: $*"
  XSPECT2_AMD_LIB_VARIANT=$v timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/cr_$n.json 2> gpurun_out/cr_$n.err || { tail -30 gpurun_out/cr_$n.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/cr_$n.json'));r=d['roofline'];print('step %.2f ms  probe %.2f ms  frac %.3f'%(d['ms_per_step'],r['probe_ms_avg'],r['frac']))"
}
run f100_cr "" --workload mlst --mlst-foreign 1.0
run f100_off nocr --workload mlst --mlst-foreign 1.0
run f90_cr "" --workload mlst --mlst-foreign 0.9
run f90_off nocr --workload mlst --mlst-foreign 0.9
