# New round-2 parity tests first (verbose), then the whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02t; mkdir -p $F
echo "== new"; timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "over_mall or mixed_streams" > $F/new.log 2>&1 || { tail -40 $F/new.log; exit 12; }
grep -E "PASS|FAIL|passed|failed" $F/new.log | tail -6
echo "== all"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 13; }
tail -2 $F/all.log
