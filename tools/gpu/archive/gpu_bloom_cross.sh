# Member-fraction crossover of the rbloom probe paths: gather (PART=0) vs partitioned forced (PART=2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for frac in ${FRACS:-0.1 0.2 0.25 0.3 0.5 1.0}; do
  for mode in 0 2; do
    XSPECT2_AMD_BLOOM_PART=$mode timeout -k 10 300 python bench.py --workload genus --no-cpu-baseline --no-host-path --steps 10 --warmup 3 --genus-filter-frac $frac > gpurun_out/bc.json 2> gpurun_out/bc.err || { tail -20 gpurun_out/bc.err; exit 8; }
    python3 -c "import json;d=json.load(open('gpurun_out/bc.json'));r=d['roofline'];print('filter frac $frac part $mode: member fraction %.3f probe %.2f ms' % (d['config']['member_fraction'], r['probe_ms_avg']))"
  done
done
