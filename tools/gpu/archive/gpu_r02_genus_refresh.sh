# Genus refresh at HEAD: bench line (with CPU baseline and host path) and kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
F=gpurun_out/r02genus; rm -rf $F; mkdir -p $F
timeout -k 10 600 python bench.py --workload genus > $F/bench_genus.json 2> $F/bench_genus.err || { tail -30 $F/bench_genus.err; exit 13; }
python3 -c "import json;d=json.load(open('$F/bench_genus.json'));print(d['value'], d['ms_per_step'], d['roofline']['probe_ms_avg'], d['roofline']['frac'], d['cpu_baseline']['value'], d['cpu_baseline']['parity_sample_mismatches'])"
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$F/trace_genus" -o run -- python3 "$R/bench.py" --workload genus --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > "$R/$F/trace_genus.json" 2> "$R/$F/trace_genus.err" || { tail -20 "$R/$F/trace_genus.err"; exit 21; }
cd "$R" && python3 tools/kstats.py $F/trace_genus/run_kernel_stats.csv | sed -n '2,5p'
