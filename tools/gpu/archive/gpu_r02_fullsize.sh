# Full-size (BASELINE config 2) property tests: both device probe paths agree on
# 1 M reads, totals, no false negatives, oracle sample.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02full; rm -rf $F; mkdir -p $F
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 300 --timeout-method thread > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
grep -E "PASS|FAIL|passed|failed" $F/tests.log | tail -4
