# Config 5 rehearsal: predict_docs_sharded over 2 ranks on one GPU (gloo), checked
# against one process; the world-1 RCCL device-path test.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03d; mkdir -p $F
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_distributed.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
grep -E "PASS|FAIL|passed|failed" $F/tests.log | tail -5
R=/tmp/r03docs
timeout -k 10 600 python -u tools/sharded_classify.py docs-setup --root $R --reads 300000 > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 12; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 13; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 tools/sharded_classify.py docs-shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 14; }
timeout -k 10 120 python tools/sharded_classify.py docs-check --root $R > $F/check.json 2>&1 || { cat $F/check.json; exit 15; }
cat $F/check.json
