# How each partitioned-COBS pass scales with the CUs it gets (hipExtStreamCreateWithCUMask
# quarters of every XCD; passes still serial): species bench, per-pass live times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03cu; mkdir -p $F
for cfg in "0 0" "4 0" "3 0" "2 0" "1 0" "0 3" "0 2" "0 1"; do
  set -- $cfg
  XSPECT2_AMD_CP_LQ=$1 XSPECT2_AMD_CP_BQ=$2 timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-host-path --no-cpu-baseline --no-e2e > $F/b_$1_$2.json 2> $F/b_$1_$2.err || { tail -20 $F/b_$1_$2.err; exit 11; }
  python -c "import json; d=json.load(open('$F/b_$1_$2.json')); r=d['roofline']; print('LQ=$1 BQ=$2', round(d['ms_per_step'],3), {k: round(v,3) for k, v in r['pass_ms_avg'].items()})"
done
