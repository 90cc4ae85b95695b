# A/B of XSPECT2_AMD_WIDE_P on wide classic banks:  bash tools/gpu/gpu_wide_ab.sh "1000 300" "1 2 4"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for d in $1; do
  for p in $2; do
    echo "== D=$d P=$p"
    XSPECT2_AMD_WIDE_P=$p timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --docs $d --genome-len 1000000 > gpurun_out/wide_${d}_$p.json 2> gpurun_out/wide_${d}_$p.err || { tail -30 gpurun_out/wide_${d}_$p.err; exit 13; }
    python -c "import json;d=json.load(open('gpurun_out/wide_${d}_$p.json'));r=d['roofline'];print('value %.3e probes/s  step %.2f ms  probe %.2f ms  %.0f GB/s frac %.3f'%(d['value'],d['ms_per_step'],r['probe_ms_avg'],r['achieved'],r['frac']))"
  done
done
