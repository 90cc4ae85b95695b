# Kernel trace of the species bench on the partitioned COBS path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F; rm -rf $F/trace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace_bench.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_bench.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py $F/trace/run_kernel_stats.csv
