# Round-2 refresh at HEAD (part 1): smoke, every -m gpu test, species and genus bench lines,
# rocprofv3 kernel traces of both.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
F=gpurun_out/r02final; rm -rf $F; mkdir -p $F
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -30 $F/smoke.log; exit 11; }
tail -1 $F/smoke.log
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 12; }
tail -1 $F/gpu_tests.log
for w in species genus; do
  echo "== bench $w"; timeout -k 10 600 python bench.py --workload $w > $F/bench_$w.json 2> $F/bench_$w.err || { tail -30 $F/bench_$w.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/bench_$w.json'));print(d['value'], d['ms_per_step'], d['roofline']['probe_ms_avg'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['parity_sample_mismatches'])"
done
for w in species genus; do
  echo "== trace $w"
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$F/trace_$w" -o run -- python3 "$R/bench.py" --workload $w --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$R/$F/trace_$w.json" 2> "$R/$F/trace_$w.err" || { tail -20 "$R/$F/trace_$w.err"; exit 21; }
  cd "$R" && python3 tools/kstats.py $F/trace_$w/run_kernel_stats.csv | sed -n '2,6p'
done
