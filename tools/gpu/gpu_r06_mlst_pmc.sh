# The MLST locus probe's PMC passes and kernel statistics (round 6: the
# bit-sliced probe_cobs_vslice replaced probe_cobs_wide on MLST loci).
#   bash tools/gpu/gpu_r06_mlst_pmc.sh
# Outputs under gpurun_out/vs3/ (copied to profiles/r06_pmc_mlst_vslice.json,
# profiles/r06_mlst_vslice_kernel_stats.csv; the same passes over the previous
# kernel gave profiles/r06_pmc_mlst_wide.json).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/vs3
mkdir -p $P
B="bench.py --workload mlst --steps 2 --warmup 1 --no-cpu-baseline --no-host-path --no-e2e"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" "SQ_WAIT_ANY TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "probe_cobs" --output-format csv -d $P/p$i -o run -- python3 $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done
python3 tools/pmc_kernels.py $P "mlst locus probe, probe_cobs_vslice<31,3>, 1 M reads" $P/pmc.json > /dev/null
rm -rf $P/p*/
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$P/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload mlst --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > "$GRAFT_REPO_ROOT/$P/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$P/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$P/trace.err"; exit 31; }
cd "$GRAFT_REPO_ROOT" && f=$(find $P/trace -name "*kernel_stats.csv" | head -1) && cp $f $P/kernel_stats.csv && rm -rf $P/trace
head -3 $P/kernel_stats.csv | cut -d, -f1-4
