# Round 5, last check at HEAD: smoke, the whole GPU suite and the default
# bench line (what the driver runs at round end).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05last; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
python3 -c "import json; d=json.loads(open('$F/species.json').read().strip().splitlines()[-1]); print(d['build_id'], d['value'], d['ms_per_step'], d['checks']['ok'], d['roofline']['frac'], d['roofline'].get('traffic_frac'))"
