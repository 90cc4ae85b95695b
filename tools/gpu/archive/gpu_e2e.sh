# GPU tests, then the end-to-end file -> hits timing (native reader)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 5; }
tail -1 gpurun_out/gpu_tests.log
echo "== e2e"
timeout -k 10 600 python tools/bench_e2e.py --dir /tmp > gpurun_out/e2e.json 2> gpurun_out/e2e.err || { tail -20 gpurun_out/e2e.err; exit 6; }
cat gpurun_out/e2e.json
