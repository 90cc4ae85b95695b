# Round 4: the device reader's pread threads per window load
# (XSPECT2_AMD_FX_LOAD_THREADS) A/B on the e2e timing, ring default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04q; mkdir -p $F
for T in 3 6 10 14; do
  XSPECT2_AMD_FX_LOAD_THREADS=$T timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen_$T.json 2> $F/gen_$T.err || { tail -30 $F/gen_$T.err; exit 21; }
  echo "threads $T: $(cat $F/gen_$T.json)"
done
for T in 6 14; do
  XSPECT2_AMD_FX_LOAD_THREADS=$T timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/genb_$T.json 2> $F/genb_$T.err || { tail -30 $F/genb_$T.err; exit 22; }
  echo "threads $T again: $(cat $F/genb_$T.json)"
done
