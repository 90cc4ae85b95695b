# Round 5: GPU suite, smoke and default bench line on the rebuilt library
# (classify_* release their banks; header helpers inline; drain guard in query_host).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05k; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
timeout -k 10 600 python -u bench.py --rccl-world1 --steps 3 --warmup 1 --no-host-path --no-e2e --no-cpu-baseline > $F/species_rccl1.json 2> $F/species_rccl1.err || { tail -30 $F/species_rccl1.err; exit 13; }
python3 - <<'PY'
import json
for f in ("species", "species_rccl1"):
    d = json.loads(open(f"gpurun_out/r05k/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], d["checks"]["ok"], r["frac"], r.get("traffic_frac"), (r.get("lookup_l2") or {}).get("frac"), (r.get("lookup_l2") or {}).get("kernel"))
PY
# host only: first-touch cost with and without transparent huge pages (tools/thp_probe.py)
timeout -k 10 120 python3 tools/thp_probe.py > gpurun_out/r05k/thp.json && cat gpurun_out/r05k/thp.json
