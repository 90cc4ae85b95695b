# Timing split of the partitioned rbloom probe (debug knobs skip work; results wrong by design).
# lookup: 1 no miss stores, 2 no filter loads, 4 no entry loads; bucket: 32 no hashing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for dbg in ${DBGS:-0 32 1 33}; do
  XSPECT2_AMD_BLOOM_DBG=$dbg timeout -k 10 300 python bench.py --workload genus --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bpd.json 2> gpurun_out/bpd.err || { tail -20 gpurun_out/bpd.err; exit 8; }
  python3 -c "import json;d=json.load(open('gpurun_out/bpd.json'));r=d['roofline'];print('dbg $dbg: probe %.2f ms' % (r['probe_ms_avg'],))"
done
P=gpurun_out/bpq; rm -rf $P; mkdir -p $P
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "bloom_bucket" --output-format csv -d $P/p$i -o run -- python3 bench.py --workload genus --no-cpu-baseline --steps 2 --warmup 1 > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU
SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_WR
GROUPS
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/bpq/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        if int(r['Grid_Size']) > 30_000_000:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(k, ' '.join('%.4g' % x for x in v[:3]))
PY
