# Resolve with two ds_and_b64 per row (XSPECT2_AMD_CP_R64=1) vs four ds_and_b32: parity, then interleaved lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03r64; mkdir -p $F
XSPECT2_AMD_CP_R64=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "partitioned or padding or entry_width or mixed_streams" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
}
for rep in 1 2; do
  run b32_$rep XSPECT2_AMD_CP_R64=0
  run b64_$rep XSPECT2_AMD_CP_R64=1
done
