# Round 4: warm the parse stream's device-to-host path on a helper thread:
# reader GPU tests, then the bench's first end-to-end call traced, with and
# without the warm-up.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04dd; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_pipeline.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -1 $F/tests.log
for W in 1 0; do
  XSPECT2_AMD_FX_WARM_D2H=$W XSPECT2_AMD_FASTX_TRACE=1 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-host-path --steps 3 --warmup 1 > $F/b_$W.json 2> $F/b_$W.err || { tail -30 $F/b_$W.err; exit 12; }
  python3 -c "
import json; d=json.loads([l for l in open('$F/b_$W.json') if l.startswith('{')][-1])
print('warm=$W', round(d['roofline']['probe_ms_avg'],2), {k:(round(v['ms'],2), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
  grep "copy phase" $F/b_$W.err | head -3
done
