# Round 4: run copies with coalesced bounds (64 runs per wave): reader GPU
# tests, e2e at 1 M and 12.5 M reads (untraced), then a kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04w; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_pipeline.py tests/test_gpu_filter.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen1m.json 2> $F/gen1m.err || { tail -30 $F/gen1m.err; exit 21; }
echo "1M: $(cat $F/gen1m.json)"
timeout -k 10 600 python -u tools/e2e_stall.py --modes gen --reps 3 --reads 12500000 > $F/gen12m.json 2> $F/gen12m.err || { tail -30 $F/gen12m.err; exit 22; }
echo "12.5M: $(cat $F/gen12m.json)"
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/e2e_stall.py" --modes gen --reps 2 --reads 12500000 > "$GRAFT_REPO_ROOT/$F/trace_gen.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 15; }
cd "$GRAFT_REPO_ROOT" && f=$(find $F/trace -name "*kernel_stats.csv" | head -1) && cp $f $F/kernel_stats.csv && rm -f $(find $F/trace -name "*kernel_trace.csv")
python3 -c "
import csv
for r in list(csv.DictReader(open('$F/kernel_stats.csv')))[:14]: print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1e3,1))"
