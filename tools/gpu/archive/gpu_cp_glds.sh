# Partitioned COBS lookup: LDS-DMA row gathers (global_load_lds_dwordx4 into per-wave slots)
# vs the default register gathers, same box (XSPECT2_AMD_CP_LOOKUP 0 / 3 u8 / 4 u4 / 5 u16).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02glds; mkdir -p $F
for v in 0 3 4 5 0; do
  XSPECT2_AMD_CP_LOOKUP=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-host-path --cpu-seconds 2 > $F/v$v.json 2> $F/v$v.err || { tail -20 $F/v$v.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/v$v.json'));c=d['cpu_baseline'] or {};print('v$v', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
done
