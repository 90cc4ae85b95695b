# Round 5, first box: smoke, the GPU suite after the knob removal and the
# hit-copy thread, the default bench line, the config-3 N=2 shared-GPU
# rehearsal of bench.py (12.5M reads per rank, per-rank self-checks), and the
# end-to-end trace (kernel + memory-copy trace of the file -> totals leg).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05a; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-400 $F/species.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $F/n2_config3.json 2> $F/n2_config3.err || { tail -30 $F/n2_config3.err; exit 13; }
cut -c1-400 $F/n2_config3.json
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d "$GRAFT_REPO_ROOT/$F/e2e_trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/e2e_trace.py" > "$GRAFT_REPO_ROOT/$F/e2e_trace.json" 2> "$GRAFT_REPO_ROOT/$F/e2e_trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/e2e_trace.err"; exit 14; }
cd "$GRAFT_REPO_ROOT" && python3 tools/e2e_trace_table.py $F/e2e_trace $F/e2e_trace.json > $F/e2e_table.txt 2>&1; head -80 $F/e2e_table.txt
