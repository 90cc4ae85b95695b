# rbloom partitioned probe without the per-call miss-byte memset (the resolve clears what the lookup set):
# whole GPU suite, then genus lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03miss; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 11; }
tail -1 $F/all.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --workload genus --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/g$rep.json 2> $F/g$rep.err || { tail -20 $F/g$rep.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/g$rep.json'));r=d['roofline'];print('g$rep', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()}, d['cpu_baseline'])"
done
