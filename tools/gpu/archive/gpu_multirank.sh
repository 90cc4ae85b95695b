# Rehearse the N>1 bench path on a one-GPU box: 2 ranks share cuda:0
# (XSPECT_BENCH_SHARE_GPU=1: gloo collectives through host copies).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
export XSPECT_BENCH_SHARE_GPU=1
for w in species multigenus genus; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --workload $w \
      > gpurun_out/multirank_$w.json 2> gpurun_out/multirank_$w.err || { tail -30 gpurun_out/multirank_$w.err; exit 7; }
  cat gpurun_out/multirank_$w.json
done
