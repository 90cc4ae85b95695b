# Round 4: bench.py's own launcher on the one-GPU box (no torchrun): the
# shared-GPU N=2 species and multigenus lines (gloo), whether RCCL lets two
# ranks share the device, the distributed GPU tests, the config-5 N=2
# rehearsal with output sharded by reads, then the genus PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04launch; mkdir -p $F
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --steps 5 --warmup 2 --launch-timeout 360 > $F/species_n2.json 2> $F/species_n2.err || { tail -30 $F/species_n2.err; exit 10; }
cut -c1-600 $F/species_n2.json
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 -u bench.py --gpus 2 --workload multigenus --steps 5 --warmup 2 --launch-timeout 360 > $F/multigenus_n2.json 2> $F/multigenus_n2.err || { tail -30 $F/multigenus_n2.err; exit 11; }
cut -c1-300 $F/multigenus_n2.json
timeout -k 10 120 python3 -u -c "
import sys; sys.path.insert(0, '.')
import bench
sys.exit(bench.launch_ranks(2, [sys.executable, 'tools/rccl_share_probe.py'], 90))
" > $F/rccl_share.txt 2>&1; rc=$?; echo "rccl_share exit $rc" >> $F/rccl_share.txt
tail -5 $F/rccl_share.txt
[ $rc -le 2 ] || exit 13
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_distributed.py tests/test_gpu_doc_slices.py > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 14; }
grep -E "passed|failed" $F/tests.log | tail -2
R=/tmp/r04docs
timeout -k 10 600 python -u tools/sharded_classify.py docs-setup --root $R --reads 300000 > $F/dsetup.log 2>&1 || { tail -30 $F/dsetup.log; exit 15; }
timeout -k 10 300 python -u tools/sharded_classify.py docs-single --root $R > $F/dsingle.log 2>&1 || { tail -30 $F/dsingle.log; exit 16; }
XSPECT_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29535 tools/sharded_classify.py docs-shard --root $R > $F/dshard.log 2>&1 || { tail -30 $F/dshard.log; exit 17; }
timeout -k 10 120 python tools/sharded_classify.py docs-check --root $R --world 2 > $F/docs_check.json 2>&1 || { cat $F/docs_check.json; exit 18; }
cat $F/docs_check.json
bash tools/gpu/gpu_r04_genus_pmc.sh > $F/genus_pmc.txt 2>&1 || { tail -20 $F/genus_pmc.txt; exit 19; }
tail -8 $F/genus_pmc.txt
