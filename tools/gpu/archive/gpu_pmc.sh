# PMC passes (one group per rocprofv3 run) over a short bench; summaries to gpurun_out/pmc/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmc
mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 400 rocprofv3 --pmc $grp --output-format csv -d $P/p$i -o run -- python $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_INT64
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum
TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
FETCH_SIZE
GROUPS
python3 tools/pmc_summary.py $P > $P/summary.txt && cat $P/summary.txt
