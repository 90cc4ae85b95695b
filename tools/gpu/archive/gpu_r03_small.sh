# Small host calls (query_small): their parity tests, the whole GPU suite (the
# probe kernels' unit grab became a runtime field), the latency tool and the
# default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03sm2; mkdir -p $F
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_small_calls.py > $F/small.log 2>&1 || { tail -40 $F/small.log; exit 11; }
grep -E "passed|failed" $F/small.log | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 12; }
tail -2 $F/all.log
timeout -k 10 300 python -u tools/latency.py > $F/lat.json 2> $F/lat.err || { tail -20 $F/lat.err; exit 13; }
grep -v amdgpu.ids $F/lat.err | tail -8
timeout -k 10 600 python -u bench.py --no-e2e > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 14; }
cut -c1-260 $F/species.json
