# Round 4: the device reader's loader queue (two windows ahead): reader GPU
# tests (both stream modes), e2e at 1 M and 12.5 M reads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04aa; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_pipeline.py tests/test_gpu_filter.py tests/test_gpu_distributed.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
XSPECT2_AMD_FX_ONE_STREAM=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py > $F/tests_one.log 2>&1 || { tail -40 $F/tests_one.log; exit 12; }
tail -1 $F/tests_one.log
timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen1m.json 2> $F/gen1m.err || { tail -30 $F/gen1m.err; exit 21; }
echo "1M: $(cat $F/gen1m.json)"
timeout -k 10 600 python -u tools/e2e_stall.py --modes gen --reps 3 --reads 12500000 > $F/gen12m.json 2> $F/gen12m.err || { tail -30 $F/gen12m.err; exit 22; }
echo "12.5M: $(cat $F/gen12m.json)"
