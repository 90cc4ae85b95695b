# Round 4, first full pass: the whole GPU suite at HEAD, then the launcher /
# distributed rehearsals and genus PMC (gpu_r04_launch.sh), then the device
# reader's per-window trace of the end-to-end legs (tools/fx_dev_trace.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04a; mkdir -p $F
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $F/smoke.log 2>&1 || { tail -20 $F/smoke.log; exit 9; }
tail -1 $F/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 8; }
tail -2 $F/all.log
bash tools/gpu/gpu_r04_launch.sh || exit $?
timeout -k 10 300 python -u tools/fx_dev_trace.py --bank --reads 1000000 --batch-mb 256 > $F/fxtrace.json 2> $F/fxtrace.err || { tail -30 $F/fxtrace.err; exit 20; }
grep -v amdgpu.ids $F/fxtrace.err | tail -30; cat $F/fxtrace.json
