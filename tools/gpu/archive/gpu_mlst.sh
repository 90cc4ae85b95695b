# parity tests, then the MLST workload (slot kernel) and a kernel trace of it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 5; }
tail -1 gpurun_out/gpu_tests.log
echo "== bench mlst"
timeout -k 10 600 python bench.py --workload mlst > gpurun_out/bench_mlst.json 2> gpurun_out/bench_mlst.err || { tail -20 gpurun_out/bench_mlst.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/bench_mlst.json'));r=d['roofline'];c=d['cpu_baseline'] or {};print('value %.3e probes/s  step %.2f ms  probe %.2f ms x%d  %.0f GB/s frac %.3f  cpu %.3e mism %s'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['probe_launches'],r['achieved'],r['frac'],c.get('value',0),c.get('parity_sample_mismatches')))"
echo "== trace mlst"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_mlst -o run -- python bench.py --workload mlst --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/trace_mlst.json 2> gpurun_out/trace_mlst.err || { tail gpurun_out/trace_mlst.err; exit 4; }
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/trace_mlst/run_kernel_stats.csv')))
for r in rows[:9]:
    print('%-60s %4s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
"
