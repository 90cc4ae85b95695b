# rbloom probe: all K loads at once vs two-phase (first SPLIT bits, then the rest)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for frac in 1.0 0.5 0.1; do
  for sp in 0 1 2 3; do
    XSPECT2_AMD_BLOOM_SPLIT=$sp timeout -k 10 300 python bench.py --workload genus --no-cpu-baseline --steps 5 --warmup 2 --genus-filter-frac $frac > gpurun_out/bl.json 2> gpurun_out/bl.err || { tail -20 gpurun_out/bl.err; exit 8; }
    python3 -c "import json;d=json.load(open('gpurun_out/bl.json'));r=d['roofline'];print('filter frac $frac split $sp: probe %.2f ms  %.3e probes/s' % (r['probe_ms_avg'], d['value']))"
  done
done
