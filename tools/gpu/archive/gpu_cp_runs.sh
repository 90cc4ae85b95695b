# Lookup: run of each entry by ballot + readlane (the window's first run, then the few runs
# starting inside it) instead of a 6-step shuffle binary search; parity, then A/B vs head.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02runs; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "partitioned or mixed_streams or over_mall or degenerate" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
  run new_$i XSPECT2_AMD_CP_LOOKUP=0
done
run new_reg XSPECT2_AMD_CP_LOOKUP=1
run new_c3 XSPECT2_AMD_CP_PERCU=3
