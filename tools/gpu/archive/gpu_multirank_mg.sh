# N=2 rehearsal of the docs-sharded (multigenus) bench on one GPU (gloo via host copies).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02mg; mkdir -p $F
export XSPECT_BENCH_SHARE_GPU=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --workload multigenus --no-host-path \
    > $F/mg.json 2> $F/mg.err || { tail -30 $F/mg.err; exit 7; }
tail -1 $F/mg.json | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('%.3e'%d['value'], round(d['ms_per_step'],2), d['config'].get('gather_dtype'))"
