# Fourth round-5 refresh at HEAD (host-side changes since gpu_r05_final3.sh:
# one HIP runtime without importing torch, the threaded repeat check; the kernels and
# hence the PMC files are unchanged): smoke, the whole GPU suite, the bench
# lines (species with host path, CPU baseline and end-to-end legs; genus; MLST;
# config 3's per-GPU shard) and a rocprofv3 kernel trace + stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05final4; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-300 $F/species.json
timeout -k 10 600 python -u bench.py --workload genus --no-e2e > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 13; }
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path --no-e2e > $F/config3_shard.json 2> $F/config3_shard.err || { tail -30 $F/config3_shard.err; exit 16; }
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > "$GRAFT_REPO_ROOT/$F/trace_bench.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 15; }
cd "$GRAFT_REPO_ROOT" && f=$(find $F/trace -name "*kernel_stats.csv" | head -1) && cp $f $F/kernel_stats.csv && rm -f $(find $F/trace -name "*kernel_trace.csv")
head -6 $F/kernel_stats.csv | cut -d, -f1-4
