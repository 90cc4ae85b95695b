# Round-3 session-2: the multi-rank library paths with the device-mode reader
# on every rank's byte range (N=2 sharded classify and docs-sharded predict,
# both ranks on cuda:0 with gloo, checked against one process), the genus and
# MLST bench lines, and a kernel trace of the default species bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03s2b; mkdir -p $F
echo "== sharded classify rehearsal (N=2, one GPU)"
R=/tmp/r03cls
timeout -k 10 600 python -u tools/sharded_classify.py setup --root $R --reads 400000 > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 13; }
timeout -k 10 300 python -u tools/sharded_classify.py single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 14; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 tools/sharded_classify.py shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 15; }
timeout -k 10 300 python tools/sharded_classify.py check --root $R --world 2 > $F/check.json 2>&1 || { cat $F/check.json; exit 16; }
cat $F/check.json; cat $F/single.log $F/shard.log | grep -E "s$|Saved" | tail -4
rm -rf $R
echo "== docs-sharded rehearsal (N=2, one GPU)"
R=/tmp/r03docs
timeout -k 10 600 python -u tools/sharded_classify.py docs-setup --root $R --reads 300000 > $F/dsetup.log 2>&1 || { tail -30 $F/dsetup.log; exit 22; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R > $F/dsingle.log 2>&1 || { tail -30 $F/dsingle.log; exit 23; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 tools/sharded_classify.py docs-shard --root $R > $F/dshard.log 2>&1 || { tail -30 $F/dshard.log; exit 24; }
timeout -k 10 120 python tools/sharded_classify.py docs-check --root $R > $F/dcheck.json 2>&1 || { cat $F/dcheck.json; exit 25; }
cat $F/dcheck.json
rm -rf $R
echo "== genus"
timeout -k 10 600 python -u bench.py --workload genus > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 31; }
cut -c1-300 $F/genus.json
echo "== mlst"
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 32; }
cut -c1-300 $F/mlst.json
echo "== kernel trace (species, no host path)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $F/trace -o run -- python bench.py --steps 10 --warmup 2 --no-host-path --no-cpu-baseline --no-e2e > $F/trace_bench.json 2> $F/trace.err || { tail -30 $F/trace.err; exit 33; }
find $F/trace -name "*kernel_stats.csv" | head -3
