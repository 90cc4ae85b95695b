# Round 4: the device reader after its changes (pooled streams, SWAR sequence
# check, host arrays behind the probe): its GPU tests, then the kernel trace
# of the end-to-end path and the per-window timeline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04f; mkdir -p $F
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_gpu_filter.py tests/test_pipeline.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
bash tools/gpu/gpu_r04_e.sh || exit $?
timeout -k 10 300 python -u tools/e2e_stall.py > $F/stall.json 2> $F/stall.err || { tail -30 $F/stall.err; exit 20; }
cat $F/stall.json
for mb in 32 16 8; do
  XSPECT2_AMD_FX_FIRST_MB=$mb timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 5 > $F/first_$mb.json 2> $F/first_$mb.err || { tail -30 $F/first_$mb.err; exit 21; }
  echo "first window $mb MiB: $(cat $F/first_$mb.json)"
done
