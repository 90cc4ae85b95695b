# Round 4: end-to-end device path A/B: parse stream priority (high default /
# low), one reader stream, and seq (no overlap) vs gen (reader thread) modes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04i; mkdir -p $F
timeout -k 10 300 python -u tools/e2e_stall.py --modes seq,gen --reps 5 > $F/base.json 2> $F/base.err || { tail -30 $F/base.err; exit 21; }
echo "high priority (default): $(cat $F/base.json)"
XSPECT2_AMD_FX_PRIORITY=low timeout -k 10 300 python -u tools/e2e_stall.py --modes seq,gen --reps 5 > $F/low.json 2> $F/low.err || { tail -30 $F/low.err; exit 22; }
echo "low priority: $(cat $F/low.json)"
XSPECT2_AMD_FX_ONE_STREAM=1 timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 5 > $F/one.json 2> $F/one.err || { tail -30 $F/one.err; exit 23; }
echo "one reader stream: $(cat $F/one.json)"
