# Round 4: H2D bandwidth from pinned memory on 1/2/4 streams (tools/h2d_bw.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
F=gpurun_out/r04l; mkdir -p $F
timeout -k 10 120 python -u tools/h2d_bw.py > $F/h2d.json 2> $F/h2d.err || { tail -20 $F/h2d.err; exit 20; }
cat $F/h2d.json
