# gpu tests, then every bench workload (default config first, with CPU baseline)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 5; }
tail -1 gpurun_out/gpu_tests.log
for w in species genus mlst multigenus; do
  echo "== bench $w"
  timeout -k 10 600 python bench.py --workload $w > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { tail -20 gpurun_out/bench_$w.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d['roofline'];c=d['cpu_baseline'] or {};print('value %.3e probes/s  step %.2f ms  probe %.2f ms x%d  %.0f GB/s frac %.3f  cpu %.3e mism %s'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['probe_launches'],r['achieved'],r['frac'],c.get('value',0),c.get('parity_sample_mismatches')))"
done
echo "== trace (species, rocprofv3 kernel stats)"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/trace.json 2> gpurun_out/trace.err || { tail gpurun_out/trace.err; exit 4; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/trace/run_kernel_stats.csv')):
    print('%-50s %4s %10.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
" | head -9
python3 -c "import json;d=json.load(open('gpurun_out/trace.json'));r=d['roofline'];print('traced: step %.2f ms probe(events) %.2f ms'%(d['ms_per_step'],r['probe_ms_avg']))"
