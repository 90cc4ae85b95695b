# Round 5: xs_query's host matrix with the recycled host pool; the whole GPU
# suite; the default bench line (host_path legs: pooled, fresh, first touch).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05c; mkdir -p $F
timeout -k 10 300 python -u tools/host_out_probe.py > $F/host_out.json 2> $F/host_out.err || { tail -20 $F/host_out.err; exit 10; }
cat $F/host_out.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-300 $F/species.json
