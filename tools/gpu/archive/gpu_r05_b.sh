# Round 5: where xs_query's host matrix time goes (first touch vs copy) after
# the hit-copy thread + prefault; the distributed and parity GPU tests that
# changed; the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05b; mkdir -p $F
timeout -k 10 300 python -u tools/host_out_probe.py > $F/host_out.json 2> $F/host_out.err || { tail -20 $F/host_out.err; exit 10; }
cat $F/host_out.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "distributed or partitioned or padding or largest" > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py --no-e2e > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-300 $F/species.json
