# COBS lookup blocks per group (XSPECT2_AMD_CP_GB: 64 default, 48, 32, 16), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03gb; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "random_configs and not bloom" > $F/parity.log 2>&1 || { tail -30 $F/parity.log; exit 12; }
XSPECT2_AMD_CP_GB=16 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "random_configs and not bloom" >> $F/parity.log 2>&1 || { tail -30 $F/parity.log; exit 12; }
grep passed $F/parity.log
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
}
for rep in 1 2; do
  for g in 64 48 32 16; do run gb${g}_$rep XSPECT2_AMD_CP_GB=$g; done
done
