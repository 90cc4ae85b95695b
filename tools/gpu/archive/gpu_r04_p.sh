# Round 4: pinned ring size A/B for the device reader's window text
# (XSPECT2_AMD_FX_RING = pieces of 4 MiB; 0 = whole-window pinned buffers):
# e2e timing per setting, then the bench end-to-end legs at the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04p; mkdir -p $F
for R in 0 8 16 32 64; do
  XSPECT2_AMD_FX_RING=$R timeout -k 10 300 python -u tools/e2e_stall.py --modes gen --reps 6 > $F/gen_$R.json 2> $F/gen_$R.err || { tail -30 $F/gen_$R.err; exit 21; }
  echo "ring $R: $(cat $F/gen_$R.json)"
done
timeout -k 10 600 python -u bench.py > $F/species.json 2> $F/species.err || { tail -30 $F/species.err; exit 12; }
python3 -c "
import json; d=json.loads([l for l in open('$F/species.json') if l.startswith('{')][-1])
print(d['value'], d['roofline']['probe_ms_avg'], {k:(round(v['ms'],2), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
