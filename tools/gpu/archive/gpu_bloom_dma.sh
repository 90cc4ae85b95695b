# rbloom partitioned lookup: LDS-DMA word gathers (XSPECT2_AMD_BLOOM_DMA 1: u16, 2: u8) x
# workgroups per CU, interleaved with the register default; genus bench, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02bdma; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload genus --steps 20 --warmup 3 --no-host-path --cpu-seconds 2 > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));c=d['cpu_baseline'] or {};print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
}
for i in 1 2; do
  run base_$i XSPECT2_AMD_BLOOM_DMA=0
  run d1c3_$i XSPECT2_AMD_BLOOM_DMA=1
  run d1c2_$i XSPECT2_AMD_BLOOM_DMA=1 XSPECT2_AMD_BLOOM_PERCU=2
  run d2c3_$i XSPECT2_AMD_BLOOM_DMA=2
  run d2c2_$i XSPECT2_AMD_BLOOM_DMA=2 XSPECT2_AMD_BLOOM_PERCU=2
  run d1c4_$i XSPECT2_AMD_BLOOM_DMA=1 XSPECT2_AMD_BLOOM_PERCU=4
done
