# Refresh the MLST (config 4) and multi-genus (config 5, N=1) bench lines with CPU baselines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in mlst multigenus; do
  timeout -k 10 600 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 6; }
  python3 -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];c=d['cpu_baseline'] or {};print('$w value %.3e probes/s  step %.2f ms  probe %.2f ms  frac %.3f  cpu %.3e mism %s'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['frac'],c.get('value',0),c.get('parity_sample_mismatches')))"
done
