# Round 4: FASTQ records found by three fused kernels: the reader's GPU tests
# and the end-to-end timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04m; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_gpu_filter.py tests/test_pipeline.py tests/test_gpu_distributed.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen.json 2> $F/gen.err || { tail -30 $F/gen.err; exit 21; }
echo "fused FASTQ records: $(cat $F/gen.json)"
grep -v amdgpu $F/gen.err | awk '/gen rep 5/,0' | grep "window\|query" | head -12
