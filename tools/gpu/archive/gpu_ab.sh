# A/B of an env knob over the default bench:  bash tools/gpu/gpu_ab.sh VAR v1 v2 ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  echo "== bench $var=$v"
  env $var=$v timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { tail -30 gpurun_out/ab_$v.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms  probe %.2f ms  %.0f GB/s frac %.3f'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['achieved'],r['frac']))"
done
