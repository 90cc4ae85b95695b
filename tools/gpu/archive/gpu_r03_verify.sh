# Re-entry check of a rebuilt container's in-tree libraries: smoke, the whole
# GPU suite and the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03verify; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 11; }
tail -2 $F/all.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
cut -c1-400 $F/species.json
