set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== randgather"; timeout -k 10 300 ./tools/randgather 16 64 200 614 2048 8192 > gpurun_out/randgather.json 2>&1 || { cat gpurun_out/randgather.json; exit 3; }
cat gpurun_out/randgather.json
echo "== tests"; timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 5; }
tail -1 gpurun_out/gpu_tests.log
echo "== trace"; timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace3 -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/trace3.json 2> gpurun_out/trace3.err || { tail gpurun_out/trace3.err; exit 4; }
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/trace3/run_kernel_stats.csv')):
    print('%-50s %4s %10.1f us' % (r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3))
" | head -8
echo "== bench"; timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail gpurun_out/bench.err; exit 6; }
cat gpurun_out/bench.json
