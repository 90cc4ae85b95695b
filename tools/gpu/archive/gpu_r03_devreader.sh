# Device-mode reader: its GPU tests (device == host batches, fallbacks, probe
# on device batches, stale batches refused), then the quick end-to-end legs of
# tools/bench_e2e.py (READS reads; progress on stderr -> $F/e2e.err).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03dr; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py > $F/tests.log 2>&1 || { tail -60 $F/tests.log; exit 11; }
grep -E "passed|failed" $F/tests.log | tail -3
[ -n "$SKIP_BENCH" ] && exit 0
timeout -k 10 600 python -u tools/bench_e2e.py --quick --reads ${READS:-1000000} --dir /tmp/e2e > $F/e2e.json 2> $F/e2e.err || { tail -30 $F/e2e.err; exit 12; }
cat $F/e2e.json
