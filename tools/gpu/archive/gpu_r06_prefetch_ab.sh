# Round 6 (a): the GPU suite after the per-handle probe options, the host
# worker pool, atomic saves and streamed doc slices; then the A/B of the
# partitioned lookup's L2 prefetch (tools/lookup_lead_ab.py) and the default
# bench line (lead 1).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r06a; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 400 python -u tools/lookup_lead_ab.py 0,1,2,4 4 > $F/lead_ab.json 2> $F/lead_ab.err || { tail -30 $F/lead_ab.err; exit 12; }
python3 -c "import json; d=json.load(open('$F/lead_ab.json')); print(json.dumps(d['five_vs_one'])); print(json.dumps(d['file_to_totals_ms'])); print(json.dumps({l: d['calls'][l]['1000000'] for l in d['calls']}))"
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 13; }
python3 -c "import json; d=json.loads(open('$F/species.json').read().strip().splitlines()[-1]); r=d['roofline']; e=d['end_to_end']['device_reader_totals']; print(d['build_id'], d['value'], d['ms_per_step'], d['checks']['ok'], r['probe_ms_avg'], r['pass_ms_avg'], e['ms'], e['ms']/r['probe_ms_avg'])"
