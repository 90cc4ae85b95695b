# LDS-DMA lookup, repeated interleaved A/B: default vs u6/u4 LDS-DMA at 2 workgroups per CU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02glds3; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run base_$i XSPECT2_AMD_CP_LOOKUP=0
  run base_c2_$i XSPECT2_AMD_CP_LOOKUP=0 XSPECT2_AMD_CP_PERCU=2
  run u6c2_$i XSPECT2_AMD_CP_LOOKUP=8 XSPECT2_AMD_CP_PERCU=2
  run u4c2_$i XSPECT2_AMD_CP_LOOKUP=4 XSPECT2_AMD_CP_PERCU=2
done
