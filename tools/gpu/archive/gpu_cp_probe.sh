# Timing probes of the partitioned COBS lookup (CK 2048): full, no store, no gather.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F
for v in 5 6 7; do
rm -rf $F/trace_v$v
cd /tmp && XSPECT2_AMD_CP_LOOKUP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace_v$v" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_v$v.json" 2> "$GRAFT_REPO_ROOT/$F/trace_v$v.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_v$v.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && echo "== v$v" && python3 tools/kstats.py $F/trace_v$v/run_kernel_stats.csv | sed -n 2,4p
done
