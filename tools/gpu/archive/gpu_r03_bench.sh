# Round 3 bench lines + kernel trace: config 2 (default, with the host path),
# genus, MLST (config 4), multigenus N=2 rehearsal (config 5, both ranks on
# cuda:0 with gloo), and a rocprofv3 kernel-trace of the default species run.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03b; mkdir -p $F
echo "== species (config 2)"
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 11; }
cut -c1-300 $F/species.json
echo "== genus"
timeout -k 10 600 python -u bench.py --workload genus > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 12; }
echo "== mlst"
timeout -k 10 600 python -u bench.py --workload mlst > $F/mlst.json 2> $F/mlst.err || { tail -30 $F/mlst.err; exit 13; }
echo "== multigenus N=2 rehearsal"
XSPECT_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --workload multigenus --no-host-path --no-cpu-baseline \
  > $F/multigenus_n2.json 2> $F/multigenus_n2.err || { tail -30 $F/multigenus_n2.err; exit 14; }
cut -c1-300 $F/multigenus_n2.json
echo "== kernel trace (species, no host path)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $F/trace -o run -- python bench.py --steps 10 --warmup 2 --no-host-path --no-cpu-baseline > $F/trace_bench.json 2> $F/trace.err || { tail -30 $F/trace.err; exit 15; }
find $F/trace -name "*kernel_stats.csv" | head -3
