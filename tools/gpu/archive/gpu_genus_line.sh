# Genus bench line (partitioned rbloom path) and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02genus; mkdir -p $F; rm -rf $F/trace
timeout -k 10 600 python bench.py --workload genus > $F/bench_genus.json 2> $F/bench_genus.err || { tail -20 $F/bench_genus.err; exit 13; }
python3 -c "import json;d=json.load(open('$F/bench_genus.json'));r=d['roofline'];print('%.3e'%d['value'], round(d['ms_per_step'],3), round(r['frac'],3), r['traffic'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload genus --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 21; }
cd "$GRAFT_REPO_ROOT" && python3 tools/kstats.py $F/trace/run_kernel_stats.csv | head -8
