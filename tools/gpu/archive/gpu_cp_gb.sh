# Lookup group size (bucket blocks a wave takes from a partition queue: 64 default, 128, 96, 32),
# parity of the partitioned tests at 128, then interleaved A/B, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02gb; mkdir -p $F
XSPECT2_AMD_CP_GB=128 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "partitioned or mixed_streams or over_mall" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run gb64_$i XSPECT2_AMD_CP_GB=64
  run gb128_$i XSPECT2_AMD_CP_GB=128
  run gb96_$i XSPECT2_AMD_CP_GB=96
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
done
