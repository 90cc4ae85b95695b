# Round 2: multi-genus (config 5, N=1) and MLST bench lines, the N=2 rehearsal
# (2 ranks share cuda:0 with gloo collectives), and the end-to-end file timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02o; mkdir -p $F
for w in multigenus mlst; do
  timeout -k 10 600 python bench.py --workload $w > $F/bench_$w.json 2> $F/bench_$w.err || { tail -20 $F/bench_$w.err; exit 6; }
  python3 -c "import json;d=json.load(open('$F/bench_$w.json'));r=d['roofline'];c=d['cpu_baseline'] or {};print('$w value %.3e probes/s  step %.2f ms  probe %.2f ms  frac %.3f  cpu %.3e mism %s'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac'],c.get('value',0),c.get('parity_sample_mismatches')))"
done
export XSPECT_BENCH_SHARE_GPU=1
for w in species multigenus; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --workload $w --no-host-path \
      > $F/multirank_$w.json 2> $F/multirank_$w.err || { tail -30 $F/multirank_$w.err; exit 7; }
  tail -1 $F/multirank_$w.json | cut -c1-200
done
unset XSPECT_BENCH_SHARE_GPU
timeout -k 10 600 python tools/bench_e2e.py --dir /tmp > $F/e2e.json 2> $F/e2e.err || { tail -20 $F/e2e.err; exit 8; }
cat $F/e2e.json
