# Kernel time split of the partitioned rbloom probe (genus bench, rocprofv3 stats).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/bp_prof" -o bp -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload genus --no-cpu-baseline --steps 5 --warmup 2 ${BP_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/bp_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/bp_prof.log"; exit 7; }
find "$GRAFT_REPO_ROOT/gpurun_out/bp_prof" -name "*kernel_stats.csv" -exec cut -c1-150 {} \;
