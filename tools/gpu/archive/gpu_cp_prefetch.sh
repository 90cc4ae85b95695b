# Lookup with the next chunk's entries loaded behind the current chunk's gathers (LOOKUP 5)
# vs the default (LOOKUP 0): parity of the partitioned tests under LOOKUP 5, then interleaved A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02pf; mkdir -p $F
XSPECT2_AMD_CP_LOOKUP=5 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "partitioned or mixed_streams or over_mall" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run l0_$i XSPECT2_AMD_CP_LOOKUP=0
  run l5_$i XSPECT2_AMD_CP_LOOKUP=5
done
run l5c3 XSPECT2_AMD_CP_LOOKUP=5 XSPECT2_AMD_CP_PERCU=3
