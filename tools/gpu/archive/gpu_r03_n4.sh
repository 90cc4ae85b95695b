# N=4 rehearsals on the one-GPU box (4 ranks on cuda:0, gloo through the host):
# config 3 sharded classify and config 5 docs-sharded predict, each checked
# against one process; plus bench.py's species N=4 path.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03n4; mkdir -p $F
R=/tmp/r03n4
timeout -k 10 600 python -u tools/sharded_classify.py setup --root $R --reads 300000 > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 11; }
timeout -k 10 300 python -u tools/sharded_classify.py single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 12; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29537 tools/sharded_classify.py shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 13; }
timeout -k 10 120 python tools/sharded_classify.py check --root $R --world 4 > $F/check_species.json 2>&1 || { cat $F/check_species.json; exit 14; }
cat $F/check_species.json
timeout -k 10 900 python -u tools/sharded_classify.py docs-setup --root $R --world 4 --reads 200000 > $F/dsetup.log 2>&1 || { tail -30 $F/dsetup.log; exit 15; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R --world 4 > $F/dsingle.log 2>&1 || { tail -30 $F/dsingle.log; exit 16; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29539 tools/sharded_classify.py docs-shard --root $R > $F/dshard.log 2>&1 || { tail -30 $F/dshard.log; exit 17; }
timeout -k 10 120 python tools/sharded_classify.py docs-check --root $R > $F/check_docs.json 2>&1 || { cat $F/check_docs.json; exit 18; }
cat $F/check_docs.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 4 --steps 5 --warmup 2 --no-host-path --no-cpu-baseline \
  > $F/bench_species_n4.json 2> $F/bench_species_n4.err || { tail -30 $F/bench_species_n4.err; exit 19; }
cut -c1-400 $F/bench_species_n4.json
