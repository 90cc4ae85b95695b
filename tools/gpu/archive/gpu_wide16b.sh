# After fixing P = 2: full GPU tests, then the wide banks and the headline.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 9; }
tail -1 gpurun_out/gpu_tests.log
: > gpurun_out/wide_banks.jsonl
for D in 200 300 600 1000 1500 2000; do
  echo "== D=$D"
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --docs $D --genome-len 1000000 > gpurun_out/wb_$D.json 2> gpurun_out/wb_$D.err || { tail -30 gpurun_out/wb_$D.err; exit 13; }
  cat gpurun_out/wb_$D.json >> gpurun_out/wide_banks.jsonl
  python -c "import json;d=json.load(open('gpurun_out/wb_$D.json'));r=d['roofline'];print('value %.3e probes/s  probe %.2f ms  frac %.3f  row %d B'%(d['value'],r['probe_ms_avg'],r['frac'],r['row_bytes']))"
done
