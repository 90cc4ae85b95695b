# Whole -m gpu suite at HEAD, then the end-to-end file -> hits / JSON timings.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03e; mkdir -p $F
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $F/all.log 2>&1 || { tail -60 $F/all.log; exit 11; }
tail -2 $F/all.log
timeout -k 10 600 python -u tools/bench_e2e.py --dir /tmp/e2e > $F/e2e.json 2> $F/e2e.err || { tail -30 $F/e2e.err; exit 12; }
cat $F/e2e.json
