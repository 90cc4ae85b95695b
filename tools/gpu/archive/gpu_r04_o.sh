# Round 4: the pinned text ring: the reader's GPU tests, the e2e timing, and
# the default bench line's end-to-end legs (first_ms).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04o; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_gpu_filter.py tests/test_pipeline.py tests/test_gpu_distributed.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen.json 2> $F/gen.err || { tail -30 $F/gen.err; exit 21; }
echo "pinned ring: $(cat $F/gen.json)"
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
python3 -c "
import json; d=json.loads([l for l in open('$F/species.json') if l.startswith('{')][-1])
print(d['value'], d['roofline']['probe_ms_avg'], {k:(round(v['ms'],2), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
