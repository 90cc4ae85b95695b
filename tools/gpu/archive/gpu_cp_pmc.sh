# PMC passes over the partitioned COBS pipeline (species bench): HBM traffic
# per kernel (FETCH_SIZE, WRITE_SIZE: separate passes) and the L2 hit rate.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmccp
rm -rf $P; mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
RX="cobs_|part_"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $P/f -o run -- python3 $B > $P/f.json 2> $P/f.err || { tail -20 $P/f.err; exit 30; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $P/w -o run -- python3 $B > $P/w.json 2> $P/w.err || { tail -20 $P/w.err; exit 31; }
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "$RX" --output-format csv -d $P/h -o run -- python3 $B > $P/h.json 2> $P/h.err || { tail -20 $P/h.err; exit 32; }
python3 tools/pmc_kernels.py $P "species, partitioned COBS" $P/pmc.json
