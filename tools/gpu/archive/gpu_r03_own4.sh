# Owner-map COBS lookup: entries per lane (XSPECT2_AMD_CP_LOOKUP 5: 6, 8: 8, 6: 10, 7: 12, 9: 14; 10: 8 with W=2048), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03own4; mkdir -p $F
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()}, 'mismatch', d['cpu_baseline'] and d['cpu_baseline'].get('parity_sample_mismatches'))"
}
for rep in 1 2; do
  run u6_$rep XSPECT2_AMD_CP_LOOKUP=5
  run u8_$rep XSPECT2_AMD_CP_LOOKUP=8
  run u10_$rep XSPECT2_AMD_CP_LOOKUP=6
  run u12_$rep XSPECT2_AMD_CP_LOOKUP=7
  run u14_$rep XSPECT2_AMD_CP_LOOKUP=9
  run u8w2k_$rep XSPECT2_AMD_CP_LOOKUP=10
done
