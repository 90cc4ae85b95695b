# Round 4: wave-cooperative FASTA line check: reader GPU tests (megabase
# lines included), then config 3's per-GPU shard end to end (bench.py legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04y; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_pipeline.py tests/test_gpu_filter.py tests/test_gpu_fullsize.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -2 $F/tests.log
timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path --no-cpu-baseline > $F/config3_e2e.json 2> $F/config3_e2e.err || { tail -30 $F/config3_e2e.err; exit 12; }
python3 -c "
import json; d=json.loads([l for l in open('$F/config3_e2e.json') if l.startswith('{')][-1])
print(d['value'], d['roofline']['probe_ms_avg'], d['end_to_end']['file_bytes'], {k:(round(v['ms'],1), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
