# Round 4 rehearsals on the one-GPU box (ranks share cuda:0 under gloo; RCCL
# refuses two ranks on one device, profiles/r04_rccl_two_ranks_one_gpu.txt):
# config 3 at N=8 with every read id repeated across shards, config 5 at N=8
# (shards by reads, all-to-all), the column-split bank at N=2, and bench.py's
# own launcher at N=8 (no torchrun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04d; mkdir -p $F
R=/tmp/r04d
timeout -k 10 600 python -u tools/sharded_classify.py setup --root $R --reads 300000 --dup > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 11; }
timeout -k 10 300 python -u tools/sharded_classify.py single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 12; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29537 tools/sharded_classify.py shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 13; }
timeout -k 10 120 python tools/sharded_classify.py check --root $R --world 8 > $F/check_species_dup_n8.json 2>&1 || { cat $F/check_species_dup_n8.json; exit 14; }
cat $F/check_species_dup_n8.json
timeout -k 10 300 python -u tools/sharded_classify.py bank-single --root $R > $F/bsingle.log 2>&1 || { tail -30 $F/bsingle.log; exit 21; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 tools/sharded_classify.py bank-shard --root $R > $F/bshard.log 2>&1 || { tail -30 $F/bshard.log; exit 22; }
timeout -k 10 120 python tools/sharded_classify.py bank-check --root $R --world 2 > $F/check_bank_n2.json 2>&1 || { cat $F/check_bank_n2.json; exit 23; }
cat $F/check_bank_n2.json
timeout -k 10 900 python -u tools/sharded_classify.py docs-setup --root $R --world 8 --reads 200000 > $F/dsetup.log 2>&1 || { tail -30 $F/dsetup.log; exit 15; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R --world 8 > $F/dsingle.log 2>&1 || { tail -30 $F/dsingle.log; exit 16; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29539 tools/sharded_classify.py docs-shard --root $R > $F/dshard.log 2>&1 || { tail -30 $F/dshard.log; exit 17; }
timeout -k 10 120 python tools/sharded_classify.py docs-check --root $R --world 8 > $F/check_docs_n8.json 2>&1 || { cat $F/check_docs_n8.json; exit 18; }
cat $F/check_docs_n8.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -u bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu-baseline --launch-timeout 540 \
  > $F/bench_species_n8.json 2> $F/bench_species_n8.err || { tail -30 $F/bench_species_n8.err; exit 19; }
cut -c1-500 $F/bench_species_n8.json
