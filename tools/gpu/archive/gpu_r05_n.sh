# Round 5: bench.py's host_path times a fresh output array's release apart
# (tools/fresh_out_probe.py found the release, not the first touch, to be
# what a fresh array costs); species (all legs) and MLST lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05n; mkdir -p $F
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
python3 - <<'PY'
import json
for f in ("species", "mlst"):
    d = json.loads(open(f"gpurun_out/r05n/{f}.json").read().strip().splitlines()[-1])
    hp = {k: {kk: round(vv, 2) for kk, vv in v.items() if kk.endswith("ms_per_step")}
          for k, v in d["host_path"].items() if isinstance(v, dict)}
    print(f, d["value"], d["ms_per_step"], d["checks"]["ok"], hp)
PY
