# One bank column-split over ranks (xs_bank_open_docs): GPU tests, then the N=2
# rehearsal (both ranks on cuda:0, gloo) of predict_bank_sharded against one process.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03bank; mkdir -p $F
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_doc_slices.py tests/test_gpu_distributed.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
grep -E "PASS|FAIL|passed|failed" $F/tests.log | tail -12
R=/tmp/r03bank
timeout -k 10 600 python -u tools/sharded_classify.py setup --root $R --reads 300000 > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 13; }
timeout -k 10 300 python -u tools/sharded_classify.py bank-single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 14; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29537 tools/sharded_classify.py bank-shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 15; }
grep -h "rank\|s$" $F/shard.log | tail -4
timeout -k 10 120 python tools/sharded_classify.py bank-check --root $R > $F/check.json 2>&1 || { cat $F/check.json; exit 16; }
cat $F/check.json
