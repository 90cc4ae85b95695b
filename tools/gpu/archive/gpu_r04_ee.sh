# Round 4: window text DMA over two copy queues (XSPECT2_AMD_FX_TWO_COPY=1)
# against one: reader tests with it on, then species and genus end-to-end legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04ee; mkdir -p $F
XSPECT2_AMD_FX_TWO_COPY=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_pipeline.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -1 $F/tests.log
for W in species genus; do
  for T in 0 1 0 1; do
    XSPECT2_AMD_FX_TWO_COPY=$T timeout -k 10 400 python -u bench.py --workload $W --no-cpu-baseline --no-host-path --steps 3 --warmup 1 > $F/${W}_$T.json 2> $F/${W}_$T.err || { tail -30 $F/${W}_$T.err; exit 12; }
    python3 -c "
import json; d=json.loads([l for l in open('$F/${W}_$T.json') if l.startswith('{')][-1])
print('$W two_copy=$T', round(d['roofline']['probe_ms_avg'],2), {k:(round(v['ms'],2), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
  done
done
