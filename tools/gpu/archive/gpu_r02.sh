# Round-2 refresh: smoke, every -m gpu test, default bench (species) and genus bench lines,
# rocprofv3 kernel trace + stats of the default bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02final
F=gpurun_out/r02final
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -30 $F/smoke.log; exit 11; }
tail -1 $F/smoke.log
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 12; }
tail -1 $F/gpu_tests.log
echo "== bench species"; timeout -k 10 600 python bench.py > $F/bench_species.json 2> $F/bench_species.err || { tail -30 $F/bench_species.err; exit 13; }
python3 -c "import json;d=json.load(open('$F/bench_species.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'], json.dumps(d['host_path']))"
echo "== bench genus"; timeout -k 10 600 python bench.py --workload genus > $F/bench_genus.json 2> $F/bench_genus.err || { tail -30 $F/bench_genus.err; exit 14; }
python3 -c "import json;d=json.load(open('$F/bench_genus.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
echo "== trace"; rm -rf $F/trace
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace_bench.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_bench.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py $F/trace/run_kernel_stats.csv | head -6
