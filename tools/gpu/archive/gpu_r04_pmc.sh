# Round-4 PMC at HEAD: the species partitioned pipeline (5 counter groups, one
# pass each) and the MLST probe's traffic (FETCH_SIZE, WRITE_SIZE passes);
# the genus pipeline's are in profiles/r04_pmc_bloompart.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmc04s
rm -rf $P; mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-e2e"
RX="cobs_|part_"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $P/p$i -o run -- python3 $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done
python3 tools/pmc_kernels.py $P "species, partitioned COBS at round-4 HEAD" $P/pmc.json > /dev/null
python3 -c "import json; d=json.load(open('$P/pmc.json')); print('species hbm_bytes_per_step', d['hbm_bytes_per_step'] / 1e9)"
M=gpurun_out/pmc04m
rm -rf $M; mkdir -p $M
BM="bench.py --workload mlst --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "probe_" --output-format csv -d $M/f -o run -- python3 $BM > $M/f.json 2> $M/f.err || { tail -20 $M/f.err; exit 31; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "probe_" --output-format csv -d $M/w -o run -- python3 $BM > $M/w.json 2> $M/w.err || { tail -20 $M/w.err; exit 32; }
python3 tools/pmc_kernels.py $M "MLST compact probe at round-4 HEAD" $M/pmc.json > /dev/null
python3 -c "import json; d=json.load(open('$M/pmc.json')); print({k: v.get('hbm_bytes') for k, v in d['kernels'].items()})"
