# rocprofv3 kernel trace + stats of the default bench (full-size launches only).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03t2; mkdir -p $F; rm -rf $F/trace
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace_bench.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_bench.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && find $F/trace -name "*.csv" && head -8 $(find $F/trace -name "*kernel_stats.csv" | head -1) | cut -c1-200
rm -f $(find $F/trace -name "*kernel_trace.csv")
