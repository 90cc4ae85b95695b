# Timing probes of the resolve (a temporary build with XSPECT2_AMD_CP_RPROBE = 1: no counting phase,
# 2: no LDS ANDs; results wrong on purpose; not in the committed source; A/B item 28).
# default, without the counting phase (1), without the LDS ANDs (2); kernel traces of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
F=gpurun_out/r02rprobe; rm -rf $F; mkdir -p $F
for pr in 0 1 2; do
  export XSPECT2_AMD_CP_RPROBE=$pr
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$F/t$pr" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-host-path --no-cpu-baseline > "$R/$F/t$pr.log" 2>&1
  cd "$R" && echo "probe $pr" && python3 tools/kstats.py $F/t$pr/run_kernel_stats.csv | grep resolve
done
