# Round 3, configs 3/5 on the box: device-resident distributed paths (world-1
# RCCL), config 3's 12.5 M-read per-GPU shard test, the N=2 torchrun rehearsal
# of the sharded classify (both ranks on cuda:0, gloo), and the config-3 shard
# bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03s; mkdir -p $F
echo "== gpu tests"
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_distributed.py tests/test_gpu_fullsize.py tests/test_gpu_models.py tests/test_gpu_parity.py tests/test_pipeline.py tests/test_gpu_known_answers.py \
  -k "docs_sharded or sharded or config3 or long_contigs or mlst or narrow or pass_stats or equals_oracle or spec_layouts or known" > $F/tests.log 2>&1 || { tail -60 $F/tests.log; exit 12; }
grep -E "PASS|FAIL|passed|failed" $F/tests.log | tail
echo "== all gpu tests"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $F/all.log 2>&1 || { tail -60 $F/all.log; exit 18; }
tail -2 $F/all.log
echo "== sharded classify rehearsal (N=2, one GPU)"
R=/tmp/r03cls
timeout -k 10 600 python -u tools/sharded_classify.py setup --root $R --reads 400000 > $F/setup.log 2>&1 || { tail -30 $F/setup.log; exit 13; }
timeout -k 10 300 python -u tools/sharded_classify.py single --root $R > $F/single.log 2>&1 || { tail -30 $F/single.log; exit 14; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 tools/sharded_classify.py shard --root $R > $F/shard.log 2>&1 || { tail -30 $F/shard.log; exit 15; }
timeout -k 10 300 python tools/sharded_classify.py check --root $R --world 2 > $F/check.json 2>&1 || { cat $F/check.json; exit 16; }
cat $F/check.json; cat $F/single.log $F/shard.log | grep -E "s$|Saved" | tail -4
echo "== bench: config 3 per-GPU shard (12.5 M reads)"
timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path > $F/bench_c3.json 2> $F/bench_c3.err || { tail -30 $F/bench_c3.err; exit 17; }
cut -c1-400 $F/bench_c3.json
echo "== bench: default (config 2) with the host path"
timeout -k 10 600 python -u bench.py > $F/bench_c2.json 2> $F/bench_c2.err || { tail -30 $F/bench_c2.err; exit 19; }
cut -c1-600 $F/bench_c2.json
