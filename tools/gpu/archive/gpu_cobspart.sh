# Partitioned COBS probe: parity tests, then species bench A/B (direct vs
# partitioned) and a kernel trace of the partitioned pipeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "classic" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -2 $F/parity.log
echo "== bench direct"; XSPECT2_AMD_COBS_PART=0 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $F/bench_direct.json 2> $F/bench_direct.err || { tail -20 $F/bench_direct.err; exit 13; }
python3 -c "import json;d=json.load(open('$F/bench_direct.json'));print(d['value'], d['ms_per_step'], d['roofline']['probe_ms_avg'])"
echo "== bench part"; XSPECT2_AMD_COBS_PART=1 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $F/bench_part.json 2> $F/bench_part.err || { tail -20 $F/bench_part.err; exit 14; }
python3 -c "import json;d=json.load(open('$F/bench_part.json'));print(d['value'], d['ms_per_step'], d['roofline']['probe_ms_avg'])"
echo "== trace"; rm -rf $F/trace
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace_bench.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace_bench.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && cut -d, -f1-4 $F/trace/run_kernel_stats.csv | head -14
