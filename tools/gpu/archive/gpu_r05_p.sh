# Round 5: pinned host memory from registered 2 MiB pages (xs::pinned_alloc)
# instead of hipHostMalloc: smoke, GPU suite, species line (host_path and
# end-to-end legs: the first call pins the reader's ring and the staging
# slots) and the MLST line (pinned outputs of 1.4 GB per locus).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05p; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 10; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
python3 - <<'PY'
import json
for f in ("species", "mlst"):
    d = json.loads(open(f"gpurun_out/r05p/{f}.json").read().strip().splitlines()[-1])
    hp = {k: {kk: round(vv, 2) for kk, vv in v.items() if kk.endswith("ms_per_step")}
          for k, v in d["host_path"].items() if isinstance(v, dict)}
    e2e = {k: v for k, v in (d.get("end_to_end") or {}).items()}
    print(f, d["value"], d["ms_per_step"], d["checks"]["ok"], hp)
    print("  e2e", json.dumps(e2e)[:900])
PY
