# LDS-DMA lookup: gathers in flight per wave (LOOKUP 0: 1, 3: 2, 4: 3, 2: 6) x workgroups
# per CU (4 waves each), padded runs, interleaved, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02inflight; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run w1c2_$i XSPECT2_AMD_CP_LOOKUP=0 XSPECT2_AMD_CP_PERCU=2
  run w1c1_$i XSPECT2_AMD_CP_LOOKUP=0 XSPECT2_AMD_CP_PERCU=1
  run w2c1_$i XSPECT2_AMD_CP_LOOKUP=3 XSPECT2_AMD_CP_PERCU=1
  run w2c2_$i XSPECT2_AMD_CP_LOOKUP=3 XSPECT2_AMD_CP_PERCU=2
  run w3c1_$i XSPECT2_AMD_CP_LOOKUP=4 XSPECT2_AMD_CP_PERCU=1
  run w6c1_$i XSPECT2_AMD_CP_LOOKUP=2 XSPECT2_AMD_CP_PERCU=1
  run reg8c2_$i XSPECT2_AMD_CP_LOOKUP=1 XSPECT2_AMD_CP_PERCU=2
done
