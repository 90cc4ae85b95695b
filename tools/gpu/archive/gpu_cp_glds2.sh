# LDS-DMA lookup sweep: unroll (3:8 4:4 5:16 6:32 7:12 8:6) x lookup workgroups per CU, same box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02glds2; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
run base XSPECT2_AMD_CP_LOOKUP=0
for v in 4 8 3 7 5 6; do for c in 2 3 4; do run v${v}_c$c XSPECT2_AMD_CP_LOOKUP=$v XSPECT2_AMD_CP_PERCU=$c; done; done
run v4_c5 XSPECT2_AMD_CP_LOOKUP=4 XSPECT2_AMD_CP_PERCU=5
run v8_c5 XSPECT2_AMD_CP_LOOKUP=8 XSPECT2_AMD_CP_PERCU=5
run base2 XSPECT2_AMD_CP_LOOKUP=0
