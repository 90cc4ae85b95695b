# Pad A/B against the previous commit's library (libxspect_hip.head.so), interleaved, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02pad2; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
  run pad4_$i XSPECT2_AMD_CP_PAD=4
  run pad1_$i XSPECT2_AMD_CP_PAD=1
done
