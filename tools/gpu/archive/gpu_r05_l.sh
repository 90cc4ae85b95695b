# Round 5: huge-page advice for pageable hit-matrix destinations (HitSink):
# host-output GPU tests, then the species and MLST bench lines (host_path legs).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05l; mkdir -p $F
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_outputs.py tests/test_gpu_parity.py -k "host or concurrent or narrow" -x -q --timeout 300 --timeout-method thread > $F/t.log 2>&1 || { tail -30 $F/t.log; exit 11; }
tail -2 $F/t.log
timeout -k 10 600 python -u bench.py --no-e2e > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 14; }
python3 - <<'PY'
import json
for f in ("species", "mlst"):
    d = json.loads(open(f"gpurun_out/r05l/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d["checks"]["ok"], {k: round(v["ms_per_step"], 2) for k, v in d["host_path"].items() if isinstance(v, dict)})
PY
