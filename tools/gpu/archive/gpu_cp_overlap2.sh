# Partitioned COBS probe with ranges overlapped on two streams (XSPECT2_AMD_CP_OVERLAP=1,
# XSPECT2_AMD_CP_RANGES = 2/3/4/6): parity, then interleaved A/B against one stream, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02ov; mkdir -p $F
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "classic_partitioned" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --cpu-seconds 2 > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));c=d['cpu_baseline'] or {};print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
}
for i in 1 2; do
  run one_$i XSPECT2_AMD_CP_OVERLAP=0
  run ov2_$i XSPECT2_AMD_CP_OVERLAP=1 XSPECT2_AMD_CP_RANGES=2
  run ov3_$i XSPECT2_AMD_CP_OVERLAP=1 XSPECT2_AMD_CP_RANGES=3
  run ov4_$i XSPECT2_AMD_CP_OVERLAP=1 XSPECT2_AMD_CP_RANGES=4
  run ov6_$i XSPECT2_AMD_CP_OVERLAP=1 XSPECT2_AMD_CP_RANGES=6
done
rm -rf $F/trace
cd /tmp && XSPECT2_AMD_CP_OVERLAP=1 XSPECT2_AMD_CP_RANGES=4 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-host-path > "$GRAFT_REPO_ROOT/$F/trace.json" 2> "$GRAFT_REPO_ROOT/$F/trace.err" || { tail -20 "$GRAFT_REPO_ROOT/$F/trace.err"; exit 21; }
