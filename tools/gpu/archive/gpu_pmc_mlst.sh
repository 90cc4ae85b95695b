# What bounds the MLST slot kernel (L2-served rows, not the HBM request ceiling)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmcm
mkdir -p $P
B="bench.py --workload mlst --steps 2 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $P/p1 -o run -- python $B > $P/p1.json 2> $P/p1.err || { tail -20 $P/p1.err; exit 30; }
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE --output-format csv -d $P/p2 -o run -- python $B > $P/p2.json 2> $P/p2.err || { tail -20 $P/p2.err; exit 31; }
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_ANY TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $P/p3 -o run -- python $B > $P/p3.json 2> $P/p3.err || { tail -20 $P/p3.err; exit 32; }
python3 tools/pmc_summary.py $P probe_cobs_slots
