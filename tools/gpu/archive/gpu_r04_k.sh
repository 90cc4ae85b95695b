# Round 4: the whole GPU suite at HEAD (sequential device reader), then the
# config-5 N=8 rehearsal (8 genus models, shards by reads, streamed merge
# checked byte for byte) and the N=8 self-launched bench (no torchrun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04k; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 11; }
tail -2 $F/all.log
R=/tmp/r04k
timeout -k 10 900 python -u tools/sharded_classify.py docs-setup --root $R --world 8 --reads 200000 > $F/dsetup.log 2>&1 || { tail -30 $F/dsetup.log; exit 15; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R --world 8 > $F/dsingle.log 2>&1 || { tail -30 $F/dsingle.log; exit 16; }
XSPECT_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
  --master-addr 127.0.0.1 --master-port 29539 tools/sharded_classify.py docs-shard --root $R > $F/dshard.log 2>&1 || { tail -30 $F/dshard.log; exit 17; }
timeout -k 10 300 python tools/sharded_classify.py docs-check --root $R --world 8 > $F/check_docs_n8.json 2>&1 || { cat $F/check_docs_n8.json; exit 18; }
cat $F/check_docs_n8.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -u bench.py --gpus 8 --steps 5 --warmup 2 --no-cpu-baseline --launch-timeout 540 \
  > $F/bench_species_n8.json 2> $F/bench_species_n8.err || { tail -30 $F/bench_species_n8.err; exit 19; }
cut -c1-400 $F/bench_species_n8.json
