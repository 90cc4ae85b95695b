# Pad A/B with the serialized LDS-DMA lookup (one gather in flight per wave), against the
# previous commit's library (libxspect_hip.head.so), interleaved, one box; parity subset first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02pad3; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "partitioned or mixed_streams or over_mall" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
  run pad4_$i XSPECT2_AMD_CP_PAD=4
  run pad1_$i XSPECT2_AMD_CP_PAD=1
  run pad4c3_$i XSPECT2_AMD_CP_PERCU=3
  run pad4c4_$i XSPECT2_AMD_CP_PERCU=4
  run pad4reg_$i XSPECT2_AMD_CP_LOOKUP=1
done
