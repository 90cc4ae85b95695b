# Round 4: do the reader's and the bank's streams share hardware queues
# (GPU_MAX_HW_QUEUES, 4 by default)?  The end-to-end device path with 4, 8
# and 16 queues.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04h; mkdir -p $F
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 5 > $F/q$q.json 2> $F/q$q.err || { tail -30 $F/q$q.err; exit 21; }
  echo "hw queues $q: $(cat $F/q$q.json)"
done
XSPECT2_AMD_FX_ONE_STREAM=1 timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 5 > $F/one_stream.json 2> $F/one_stream.err || { tail -30 $F/one_stream.err; exit 22; }
echo "one reader stream, hw queues 4: $(cat $F/one_stream.json)"
