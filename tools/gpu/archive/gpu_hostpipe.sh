# Host batches staged in chunks, overlapped with the probe: parity + bench host path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/par_hp.log 2>&1 || { tail -40 gpurun_out/par_hp.log; exit 9; }
echo "parity: $(tail -1 gpurun_out/par_hp.log)"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/hp_species.json 2> gpurun_out/hp_species.err || { tail -30 gpurun_out/hp_species.err; exit 13; }
python -c "import json;d=json.load(open('gpurun_out/hp_species.json'));print(d['ms_per_step'], json.dumps(d['host_path']))"
