# Round 4: allocation costs (tools/alloc_cost.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
F=gpurun_out/r04n; mkdir -p $F
timeout -k 10 120 python -u tools/alloc_cost.py > $F/alloc.json 2> $F/alloc.err || { tail -20 $F/alloc.err; exit 20; }
cat $F/alloc.json
