# Round-3 GPU tests: the new/changed files first (verbose), then the whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03t; mkdir -p $F
NEW=${NEW:-"tests/test_gpu_known_answers.py tests/test_integration_stub.py"}
echo "== new: $NEW"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $NEW ${NEWK:+-k "$NEWK"} > $F/new.log 2>&1 || { tail -60 $F/new.log; exit 12; }
grep -E "PASS|FAIL|passed|failed" $F/new.log | tail -12
echo "== all"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -60 $F/all.log; exit 13; }
tail -3 $F/all.log
