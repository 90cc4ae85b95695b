# Selected GPU tests (pass a -k expression as $1), verbose.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/q/tests.log 2>&1 || { tail -40 gpurun_out/q/tests.log; exit 12; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/q/tests.log | tail -12
