# Partitioned rbloom lookup: entries in flight per lane (4/8/16) A/B, plus the direct probe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for frac in 1.0 0.1; do
  for u in 4 8 16; do
    for dbg in 0 1; do
    XSPECT2_AMD_BLOOM_DBG=$dbg XSPECT2_AMD_BLOOM_UNROLL=$u timeout -k 10 300 python bench.py --workload genus --no-cpu-baseline --steps 5 --warmup 2 --genus-filter-frac $frac > gpurun_out/bpu.json 2> gpurun_out/bpu.err || { tail -20 gpurun_out/bpu.err; exit 8; }
    python3 -c "import json;d=json.load(open('gpurun_out/bpu.json'));r=d['roofline'];print('frac $frac unroll $u dbg $dbg: probe %.2f ms' % (r['probe_ms_avg'],))"
    done
  done
done
