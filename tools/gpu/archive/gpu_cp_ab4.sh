# Partitioned COBS probe A/B round 4: pipelined block ranges (XSPECT2_AMD_CP_SUB) x lookup blocks per CU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "classic or mixed_streams" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), d['cpu_baseline'] and d['cpu_baseline'].get('parity_sample_mismatches'))"
}
run direct XSPECT2_AMD_COBS_PART=0
for sub in 1 2 3 4 6; do run sub$sub XSPECT2_AMD_CP_SUB=$sub; done
for c in 2 4; do run sub3_c$c XSPECT2_AMD_CP_SUB=3 XSPECT2_AMD_CP_PERCU=$c; done
run sub3_v1 XSPECT2_AMD_CP_SUB=3 XSPECT2_AMD_CP_LOOKUP=1
