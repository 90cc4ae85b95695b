# Partitioned COBS queries without the direct probe's unit map: whole GPU suite, bench lines, kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03nounits; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 11; }
tail -1 $F/all.log
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/b$rep.json 2> $F/b$rep.err || { tail -20 $F/b$rep.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/b$rep.json'));r=d['roofline'];print('b$rep', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 15; }
cd "$GRAFT_REPO_ROOT" && rm -f $(find $F/trace -name "*kernel_trace.csv") && ls $F/trace
