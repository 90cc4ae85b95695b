# Partitioned COBS probe A/B round 2: bucket block size x lookup variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02cp; mkdir -p $F
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "classic" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
run direct XSPECT2_AMD_COBS_PART=0
for ck in 1024 2048; do for v in 0 2 4 5; do run ck${ck}_v$v XSPECT2_AMD_CP_CK=$ck XSPECT2_AMD_CP_LOOKUP=$v; done; done
