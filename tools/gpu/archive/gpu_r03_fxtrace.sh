# Device-mode reader phase trace (tools/fx_dev_trace.py) on one MI355X box,
# at each batch size of MBS.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03fx; mkdir -p $F
for mb in ${MBS:-256 64}; do
  timeout -k 10 300 python -u tools/fx_dev_trace.py ${BANK:+--bank} --reads ${READS:-1000000} --batch-mb $mb > $F/trace_$mb.json 2> $F/trace_$mb.err || { tail -30 $F/trace_$mb.err; exit 12; }
  grep -v amdgpu.ids $F/trace_$mb.err | tail -12; cat $F/trace_$mb.json
done
