# Targeted GPU tests for the round-2 changes, then the full -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r02
F=gpurun_out/r02
echo "== new tests"; timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "mixed_streams or odd_byte" tests/test_pipeline.py > $F/new_tests.log 2>&1 || { tail -40 $F/new_tests.log; exit 12; }
tail -3 $F/new_tests.log
echo "== gpu tests"; timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 13; }
tail -3 $F/gpu_tests.log
