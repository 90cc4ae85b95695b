# Round 5, late: the N>1 paths on the current library (the load no longer
# imports torch itself): the config-3 N=2 shared-GPU rehearsal (gloo, 12.5M
# reads per rank, per-rank self-checks) and the one-rank RCCL group line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05w; mkdir -p $F
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 900 python -u bench.py --gpus 2 --steps 5 --warmup 2 > $F/n2_config3.json 2> $F/n2_config3.err || { tail -30 $F/n2_config3.err; exit 13; }
timeout -k 10 600 python -u bench.py --rccl-world1 --reads 12500000 --steps 3 --warmup 1 --no-host-path --no-e2e --no-cpu-baseline > $F/rccl1_config3.json 2> $F/rccl1_config3.err || { tail -30 $F/rccl1_config3.err; exit 14; }
python3 - <<'PY'
import json
for f in ("n2_config3", "rccl1_config3"):
    d = json.loads(open(f"gpurun_out/r05w/{f}.json").read().strip().splitlines()[-1])
    print(f, d["n_gpus"], d["dist_backend"], d["config"]["workload"][:60], d["value"], d["ms_per_step"], d["checks"]["ok"],
          [{k: v for k, v in r.items() if k.endswith("mismatches")} for r in d["checks"]["per_rank"]])
PY
