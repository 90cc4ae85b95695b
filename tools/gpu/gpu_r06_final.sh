# Round 6: the one end-of-round refresh at HEAD, in two
# parts so that each stays well inside one gpurun call:
#   bash tools/gpu/gpu_r06_final.sh 1   smoke, the whole GPU suite, the bench
#        lines (species default with host path, CPU baseline and end-to-end
#        legs; genus; MLST; config 3's per-GPU shard) and a rocprofv3 kernel
#        trace + stats of the default run
#   bash tools/gpu/gpu_r06_final.sh 2   the species pipeline's PMC passes,
#        the N>1 path as the driver's 8-GPU run takes it (config 3 at N=2 with
#        both ranks on the one GPU under gloo; every collective in a one-rank
#        RCCL group), and the end-to-end kernel + copy trace
# Outputs under gpurun_out/r06final/ (copied to profiles/r06_final_*).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r06final; mkdir -p $F
line() {  # the bench line's headline fields
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['build_id'], d['value'], round(d['ms_per_step'],3), d['checks']['ok'], r.get('probe_ms_avg'), r.get('frac'), r.get('traffic_frac'))" $1
}
if [ "$1" = "1" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
  tail -1 $F/smoke.log
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
  tail -2 $F/gpu_tests.log
  timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
  line $F/species.json
  timeout -k 10 600 python -u bench.py --workload genus > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 13; }
  line $F/genus.json
  timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
  line $F/mlst.json
  timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path > $F/config3_shard.json 2> $F/config3_shard.err || { tail -30 $F/config3_shard.err; exit 15; }
  line $F/config3_shard.json
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 16; }
  cd "$GRAFT_REPO_ROOT" && f=$(find $F/trace -name "*kernel_stats.csv" | head -1) && cp $f $F/kernel_stats.csv && rm -f $(find $F/trace -name "*kernel_trace.csv")
  head -6 $F/kernel_stats.csv | cut -d, -f1-4
elif [ "$1" = "2" ]; then
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
  python3 tools/pmc_kernels.py $P "species, partitioned COBS at round-6 HEAD" $P/pmc.json > /dev/null
  python3 -c "import json; d=json.load(open('$P/pmc.json')); print('species hbm_bytes_per_step', d['hbm_bytes_per_step'] / 1e9)"
  rm -rf $P/p*/
  XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $F/n2_config3_share.json 2> $F/n2_config3_share.err || { tail -30 $F/n2_config3_share.err; exit 31; }
  timeout -k 10 600 python -u bench.py --rccl-world1 --reads 12500000 --steps 3 --warmup 1 --no-host-path --no-e2e --no-cpu-baseline > $F/rccl1_config3.json 2> $F/rccl1_config3.err || { tail -30 $F/rccl1_config3.err; exit 32; }
  timeout -k 10 600 python -u bench.py --rccl-world1 --workload multigenus --steps 3 --warmup 1 --no-host-path --no-cpu-baseline > $F/rccl1_multigenus.json 2> $F/rccl1_multigenus.err || { tail -30 $F/rccl1_multigenus.err; exit 33; }
  for f in n2_config3_share rccl1_config3 rccl1_multigenus; do
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['n_gpus'], d['dist_backend'], d['rccl_world'], d['value'], round(d['ms_per_step'],2), json.dumps(d['checks']))" $F/$f.json
  done
  cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$GRAFT_REPO_ROOT/$F/e2e_trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/e2e_trace.py" > "$GRAFT_REPO_ROOT/$F/e2e_trace.json" 2> "$GRAFT_REPO_ROOT/$F/e2e_trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/e2e_trace.err"; exit 34; }
  cd "$GRAFT_REPO_ROOT" && python3 tools/e2e_trace_table.py $F/e2e_trace $F/e2e_trace.json > $F/e2e_table.txt 2>&1; grep -E "busy|idle|probes alone|pass -1" $F/e2e_table.txt
  rm -rf $F/e2e_trace
else
  echo "usage: bash tools/gpu/gpu_r06_final.sh 1|2"; exit 2
fi
