# Round 4: ring size A/B with device sides kept across opens: e2e timing
# (8 files per process) for rings 0/32/16, and the bench's end-to-end legs
# for 0 and 32.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04s; mkdir -p $F
for R in 0 32 16; do
  XSPECT2_AMD_FX_RING=$R timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 8 > $F/gen_$R.json 2> $F/gen_$R.err || { tail -30 $F/gen_$R.err; exit 21; }
  echo "ring $R: $(cat $F/gen_$R.json)"
done
for R in 0 32; do
  XSPECT2_AMD_FX_RING=$R timeout -k 10 600 python -u bench.py > $F/species_$R.json 2> $F/species_$R.err || { tail -30 $F/species_$R.err; exit 12; }
  python3 -c "
import json; d=json.loads([l for l in open('$F/species_$R.json') if l.startswith('{')][-1])
print('ring $R', d['value'], d['roofline']['probe_ms_avg'], {k:(round(v['ms'],2), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
done
