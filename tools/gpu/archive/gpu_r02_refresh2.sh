# Round-2 refresh at HEAD (part 2): multi-genus and MLST bench lines, the N=2 rehearsal, the
# end-to-end file timing, and PMC passes (HBM traffic) of the species and genus pipelines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02o; rm -rf $F; mkdir -p $F
for w in multigenus mlst; do
  timeout -k 10 600 python bench.py --workload $w > $F/bench_$w.json 2> $F/bench_$w.err || { tail -20 $F/bench_$w.err; exit 6; }
  python3 -c "import json;d=json.load(open('$F/bench_$w.json'));r=d['roofline'];c=d['cpu_baseline'] or {};print('$w value %.3e probes/s  step %.2f ms  probe %.2f ms  frac %.3f  cpu %.3e mism %s'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac'],c.get('value',0),c.get('parity_sample_mismatches')))"
done
export XSPECT_BENCH_SHARE_GPU=1
for w in species multigenus; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --workload $w --no-host-path \
      > $F/multirank_$w.json 2> $F/multirank_$w.err || { tail -30 $F/multirank_$w.err; exit 7; }
  tail -1 $F/multirank_$w.json | cut -c1-200
done
unset XSPECT_BENCH_SHARE_GPU
timeout -k 10 600 python tools/bench_e2e.py --dir /tmp > $F/e2e.json 2> $F/e2e.err || { tail -20 $F/e2e.err; exit 8; }
echo "e2e ok"
P=gpurun_out/pmcfinal; rm -rf $P; mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "cobs_|part_" --output-format csv -d $P/p$i -o run -- python3 $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done
python3 tools/pmc_kernels.py $P "species, partitioned COBS at HEAD (padded runs, one LDS-DMA gather in flight per wave)" $P/pmc.json > /dev/null
python3 -c "import json;d=json.load(open('$P/pmc.json'));print('species hbm per step', d['hbm_bytes_per_step']/1e9)"
G=gpurun_out/pmcgenus; rm -rf $G; mkdir -p $G
BG="bench.py --workload genus --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "bloom_|part_" --output-format csv -d $G/p$i -o run -- python3 $BG > $G/p$i.json 2> $G/p$i.err || { tail -20 $G/p$i.err; exit 31; }
done
python3 tools/pmc_kernels.py $G "genus, partitioned rbloom at HEAD" $G/pmc.json > /dev/null
python3 -c "import json;d=json.load(open('$G/pmc.json'));print('genus hbm per step', d['hbm_bytes_per_step']/1e9)"
