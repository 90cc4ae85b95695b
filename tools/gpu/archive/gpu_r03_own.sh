# COBS lookup with the LDS entry -> block map (XSPECT2_AMD_CP_LOOKUP=5): parity
# of the partitioned cases, then the default bench interleaved with it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03own; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "partitioned or padding or entry_width" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
}
run base1 XSPECT2_AMD_CP_LOOKUP=0
run own1 XSPECT2_AMD_CP_LOOKUP=5
run base2 XSPECT2_AMD_CP_LOOKUP=0
run own2 XSPECT2_AMD_CP_LOOKUP=5
