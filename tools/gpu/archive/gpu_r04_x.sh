# Round 4: with the lighter parse kernels, parse ahead on a worker thread
# (XSPECT2_AMD_FX_PARSE_AHEAD=1) against parse-on-demand, at 1 M and 12.5 M reads.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04x; mkdir -p $F
for A in 0 1; do
  XSPECT2_AMD_FX_PARSE_AHEAD=$A timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen1m_$A.json 2> $F/gen1m_$A.err || { tail -30 $F/gen1m_$A.err; exit 21; }
  echo "1M ahead=$A: $(cat $F/gen1m_$A.json)"
  XSPECT2_AMD_FX_PARSE_AHEAD=$A timeout -k 10 600 python -u tools/e2e_stall.py --modes gen --reps 3 --reads 12500000 > $F/gen12m_$A.json 2> $F/gen12m_$A.err || { tail -30 $F/gen12m_$A.err; exit 22; }
  echo "12.5M ahead=$A: $(cat $F/gen12m_$A.json)"
done
