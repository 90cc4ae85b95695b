# Partitioned COBS lookup: cache-policy variants of the row gathers and the row stores
# (XSPECT2_AMD_CP_LOOKUP 0 default, 3 gather sc1, 4 gather sc0 sc1, 5 gather nt,
#  6 store sc0 sc1, 7 store sc0 sc1 nt, 8 store nt (buffer x4), 9 store sc1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02pol; mkdir -p $F
for v in 0 3 4 5 6 7 8 9; do
  XSPECT2_AMD_CP_LOOKUP=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-host-path --cpu-seconds 2 > $F/v$v.json 2> $F/v$v.err || { tail -20 $F/v$v.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/v$v.json'));c=d['cpu_baseline'] or {};print('v$v', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
done
