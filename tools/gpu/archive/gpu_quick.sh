# parity tests + kernel-trace stats of a short bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests"; timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 5; }
tail -1 gpurun_out/gpu_tests.log
echo "== trace"; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/trace.json 2> gpurun_out/trace.err || { tail gpurun_out/trace.err; exit 4; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/trace/run_kernel_stats.csv')):
    print('%-50s %4s %10.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
" | head -9
python3 -c "import json;d=json.load(open('gpurun_out/trace.json'));print('step %.2f ms value %.3e'%(d['ms_per_step'],d['value']))"
