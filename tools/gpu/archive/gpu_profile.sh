# rocprofv3 passes over the default bench (kernel trace + separate PMC passes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/prof
mkdir -p $P
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline"
echo "== trace"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python $B > $P/trace_bench.json 2> $P/trace_bench.err || { tail -20 $P/trace_bench.err; exit 21; }
echo "== pmc FETCH_SIZE"
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/pmc_fetch -o run -- python $B > $P/pmc_fetch.json 2> $P/pmc_fetch.err || { tail -20 $P/pmc_fetch.err; exit 22; }
echo "== pmc TCC"
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $P/pmc_tcc -o run -- python $B > $P/pmc_tcc.json 2> $P/pmc_tcc.err || { tail -20 $P/pmc_tcc.err; exit 23; }
echo "== pmc SQ"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $P/pmc_sq -o run -- python $B > $P/pmc_sq.json 2> $P/pmc_sq.err || { tail -20 $P/pmc_sq.err; exit 24; }
timeout -k 10 120 rocprofv3 -L > $P/counters.txt 2>&1 || true
find $P -name "*.csv" | head -30
