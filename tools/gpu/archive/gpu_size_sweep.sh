# Random-gather rate vs table size (microbenchmark) and the species probe vs bank size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 ./tools/randgather 150 300 614 1228 2456 > gpurun_out/sweep_gather.json 2> gpurun_out/sweep_gather.err || { cat gpurun_out/sweep_gather.err; exit 3; }
grep '"policy": "plain"' gpurun_out/sweep_gather.json | grep hipMalloc
for gl in 2000000 8000000 16000000; do
  echo "== D=100 genome-len $gl"
  timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --genome-len $gl > gpurun_out/sweep_$gl.json 2> gpurun_out/sweep_$gl.err || { tail -30 gpurun_out/sweep_$gl.err; exit 13; }
  python -c "import json;d=json.load(open('gpurun_out/sweep_$gl.json'));r=d['roofline'];print('value %.3e probes/s  probe %.2f ms  frac %.3f  bank %.2f GB'%(d['value'],r['probe_ms_avg'],r['frac'],d['config']['bank_device_bytes']/1e9))"
done
