# Round-3 session-2 check at HEAD: the device-reader model path in the GPU
# suite (new/changed files verbose, then everything), then the default bench
# line with its end-to-end legs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
NEW="tests/test_gpu_fastx_device.py tests/test_gpu_models.py tests/test_gpu_distributed.py" bash tools/gpu/gpu_r03_tests.sh || exit $?
F=gpurun_out/r03s2; mkdir -p $F
echo "== species bench (config 2, e2e legs)"
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 21; }
python -c "import json,sys; d=json.load(open('$F/species.json')); print(d['value'], d['ms_per_step']); print(json.dumps(d['end_to_end'], indent=1)); print(json.dumps(d['host_path']))"
