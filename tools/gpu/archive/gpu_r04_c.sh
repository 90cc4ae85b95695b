# Round 4: where the end-to-end device path waits (tools/e2e_stall.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04c; mkdir -p $F
timeout -k 10 300 python -u tools/e2e_stall.py > $F/stall.json 2> $F/stall.err || { tail -30 $F/stall.err; exit 20; }
cat $F/stall.json
