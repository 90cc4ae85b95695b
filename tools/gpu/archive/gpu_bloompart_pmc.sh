# PMC passes over the partitioned rbloom lookup kernel (genus bench).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/bpp
rm -rf $P; mkdir -p $P
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "bloom_lookup" --output-format csv -d $P/p$i -o run -- python3 bench.py --workload genus --no-cpu-baseline --steps 2 --warmup 1 > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done <<'GROUPS'
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU
TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_REQ_sum
GROUPS
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob('gpurun_out/bpp/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        if int(r['Grid_Size']) > 0:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in agg.items():
    print(k, ' '.join('%.4g' % x for x in v[:4]))
PY
