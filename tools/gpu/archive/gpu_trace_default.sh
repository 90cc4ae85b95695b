# rocprofv3 kernel trace + stats of the default bench with full-size launches only.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/final; mkdir -p $F; rm -rf $F/trace
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace_bench.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_bench.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && head -3 $F/trace/run_kernel_stats.csv | cut -c1-150 && python3 -c "import json;d=json.load(open('$F/trace_bench.json'));print('bench probe_ms_avg', d['roofline']['probe_ms_avg'])"
