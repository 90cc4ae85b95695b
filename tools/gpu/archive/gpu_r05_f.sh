# Round 5: every collective of bench.py's N>1 path in a one-rank RCCL group
# (--rccl-world1: the config-3 all-reduce, the multigenus all-to-all, the
# per-rank gathers and checks on device tensors), and the distributed GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05f; mkdir -p $F
timeout -k 10 600 python -u bench.py --rccl-world1 --reads 12500000 --steps 3 --warmup 1 --no-host-path --no-e2e --no-cpu-baseline > $F/species_rccl1.json 2> $F/species_rccl1.err || { tail -30 $F/species_rccl1.err; exit 12; }
timeout -k 10 600 python -u bench.py --rccl-world1 --workload multigenus --steps 3 --warmup 1 --no-host-path --no-cpu-baseline > $F/multigenus_rccl1.json 2> $F/multigenus_rccl1.err || { tail -30 $F/multigenus_rccl1.err; exit 13; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread > $F/dist_tests.log 2>&1 || { tail -40 $F/dist_tests.log; exit 14; }
tail -2 $F/dist_tests.log
python3 - <<'PY'
import json
for f in ("species_rccl1", "multigenus_rccl1"):
    d = json.loads(open(f"gpurun_out/r05f/{f}.json").read().strip().splitlines()[-1])
    print(f, d["dist_backend"], d["rccl_world"], d["value"], d["ms_per_step"], d["config"]["workload"][:60], json.dumps(d["checks"]))
PY
