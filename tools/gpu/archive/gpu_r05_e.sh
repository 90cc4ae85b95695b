# Round 5: the self-checks of every bench workload (genus, MLST, multigenus at
# N=1; multigenus at N=2 on the shared GPU: the exchanged-column checksums).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05e; mkdir -p $F
timeout -k 10 600 python -u bench.py --workload genus --no-e2e > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 12; }
cut -c1-200 $F/genus.json
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 13; }
cut -c1-200 $F/mlst.json
timeout -k 10 600 python -u bench.py --workload multigenus --no-host-path > $F/multigenus.json 2> $F/multigenus.err || { tail -30 $F/multigenus.err; exit 14; }
cut -c1-200 $F/multigenus.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --workload multigenus --steps 5 --warmup 2 > $F/multigenus_n2.json 2> $F/multigenus_n2.err || { tail -30 $F/multigenus_n2.err; exit 15; }
cut -c1-200 $F/multigenus_n2.json
python3 - <<'PY'
import json
for f in ("genus", "mlst", "multigenus", "multigenus_n2"):
    d = json.loads(open(f"gpurun_out/r05e/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], json.dumps(d["checks"]))
PY
