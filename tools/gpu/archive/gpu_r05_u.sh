# Round 5: the library loads torch's HIP runtime by path instead of importing
# torch: the CLI start-up probe, smoke and the whole GPU suite (device
# tensors from torch pass into the library in many of its tests).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05u; mkdir -p $F
timeout -k 10 300 python3 tools/cli_probe.py > $F/cli_after.json 2> $F/cli_after.err || { tail -20 $F/cli_after.err; exit 10; }
python3 -c "import json; print(json.load(open('$F/cli_after.json'))['best'])"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 11; }
tail -1 $F/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 12; }
tail -2 $F/gpu_tests.log
