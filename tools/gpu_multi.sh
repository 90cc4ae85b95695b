# multi-bank probe: parity tests, then the MLST step at several loci-per-launch groupings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== tests"
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -x -k "multi or compact or mlst" > gpurun_out/gpu_multi_tests.log 2>&1 || { tail -40 gpurun_out/gpu_multi_tests.log; exit 5; }
tail -1 gpurun_out/gpu_multi_tests.log
for g in ${GROUPS_LIST:-1 7 2 4}; do
  echo "== mlst group $g"
  timeout -k 10 400 python bench.py --workload mlst --mlst-group $g --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_mlst_g$g.json 2> gpurun_out/bench_mlst_g$g.err || { tail -20 gpurun_out/bench_mlst_g$g.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/bench_mlst_g$g.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms  probe %.2f ms x%d  %.0f GB/s frac %.3f'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['probe_launches'],r['achieved'],r['frac']))"
done
