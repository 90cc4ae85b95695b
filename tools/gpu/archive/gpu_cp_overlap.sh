# Kernel trace of the pipelined partitioned COBS probe (sub-batches = 3): do the passes overlap?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F; rm -rf $F/trace_sub3
cd /tmp && XSPECT2_AMD_CP_SUB=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace_sub3" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_sub3.json" 2> "$GRAFT_REPO_ROOT/$F/trace_sub3.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_sub3.err"; exit 21; }
