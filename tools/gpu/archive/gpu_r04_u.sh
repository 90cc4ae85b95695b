# Round 4: where the config-3-scale end-to-end time goes: the reader's
# per-window trace over a 12.5 M-read FASTQ, and a kernel trace of the same.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04u; mkdir -p $F
timeout -k 10 600 python -u tools/e2e_stall.py --modes gen --reps 3 --reads 12500000 > $F/gen.json 2> $F/gen.err || { tail -30 $F/gen.err; exit 21; }
echo "gen: $(cat $F/gen.json)"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/e2e_stall.py" --modes gen --reps 2 --reads 12500000 > "$GRAFT_REPO_ROOT/$F/trace_gen.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 15; }
cd "$GRAFT_REPO_ROOT" && f=$(find $F/trace -name "*kernel_stats.csv" | head -1) && cp $f $F/kernel_stats.csv && rm -f $(find $F/trace -name "*kernel_trace.csv")
cut -d, -f1-4 $F/kernel_stats.csv | cut -c1-160
