# Round-5 refresh at HEAD: smoke, the whole GPU suite, the bench lines
# (species default with host path, CPU baseline and end-to-end legs; genus;
# MLST; config 3's per-GPU shard), a rocprofv3 kernel trace + stats of the
# default run, and the species pipeline's PMC passes (one pass per counter
# group) for the line's traffic figures.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05final; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-300 $F/species.json
timeout -k 10 600 python -u bench.py --workload genus --no-e2e > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 13; }
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path --no-e2e > $F/config3_shard.json 2> $F/config3_shard.err || { tail -30 $F/config3_shard.err; exit 16; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 15; }
cd "$GRAFT_REPO_ROOT" && f=$(find $F/trace -name "*kernel_stats.csv" | head -1) && cp $f $F/kernel_stats.csv && rm -f $(find $F/trace -name "*kernel_trace.csv")
head -6 $F/kernel_stats.csv | cut -d, -f1-4
P=$F/pmc
mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-e2e"
RX="cobs_|part_"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $P/p$i -o run -- python3 $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done
python3 tools/pmc_kernels.py $P "species, partitioned COBS at round-5 HEAD" $P/pmc.json > /dev/null
python3 -c "import json; d=json.load(open('$P/pmc.json')); print('species hbm_bytes_per_step', d['hbm_bytes_per_step'] / 1e9)"
rm -rf $P/p*/ 
