# MLST (config 4) wide kernel: LDS-DMA row chunks (XSPECT2_AMD_WIDE_DMA=1) vs registers;
# compact-bank parity with DMA, then interleaved bench A/B on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02wdma; mkdir -p $F
echo "== parity"; XSPECT2_AMD_WIDE_DMA=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "compact" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload mlst --steps 5 --warmup 2 --no-host-path --cpu-seconds 2 > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));c=d['cpu_baseline'] or {};print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
}
for i in 1 2; do
  run reg_$i XSPECT2_AMD_WIDE_DMA=0
  run dma_$i XSPECT2_AMD_WIDE_DMA=1
done
