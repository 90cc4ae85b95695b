# Owner-map COBS lookup variants (XSPECT2_AMD_CP_LOOKUP 5-9, workgroups per CU), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03own3; mkdir -p $F
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
}
for rep in 1 2; do
  run v5_$rep XSPECT2_AMD_CP_LOOKUP=5
  run v6_$rep XSPECT2_AMD_CP_LOOKUP=6
  run v7_$rep XSPECT2_AMD_CP_LOOKUP=7
  run v8_$rep XSPECT2_AMD_CP_LOOKUP=8
  run v9_$rep XSPECT2_AMD_CP_LOOKUP=9
  run v5c3_$rep XSPECT2_AMD_CP_LOOKUP=5 XSPECT2_AMD_CP_PERCU=3
done
