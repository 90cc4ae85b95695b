# Partitioned rbloom probe: full GPU parity, A/B against the direct probe (default = adaptive), kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/ -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/bp_par.log 2>&1 || { tail -40 gpurun_out/bp_par.log; exit 9; }
echo "parity: $(tail -1 gpurun_out/bp_par.log)"
for frac in 1.0 0.5 0.1; do
  for mode in 0 1; do
    XSPECT2_AMD_BLOOM_PART=$mode timeout -k 10 300 python bench.py --workload genus --steps 10 --warmup 3 --genus-filter-frac $frac > gpurun_out/bp_${frac}_$mode.json 2> gpurun_out/bp.err || { tail -20 gpurun_out/bp.err; exit 8; }
    python3 -c "import json;d=json.load(open('gpurun_out/bp_${frac}_$mode.json'));r=d['roofline'];print('filter frac $frac part $mode: probe %.2f ms step %.2f ms %.3e probes/s  %s' % (r['probe_ms_avg'], d['ms_per_step'], d['value'], r['kernel'][:40]))"
  done
done
rm -rf gpurun_out/bp_prof
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/bp_prof" -o bp -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload genus --no-cpu-baseline --no-host-path --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/bp_prof.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/bp_prof.log"; exit 7; }
cd "$GRAFT_REPO_ROOT" && python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob('gpurun_out/bp_prof/*kernel_trace.csv')[0])))
big = {}
for r in rows:
    n = r['Kernel_Name']
    if any(x in n for x in ('bloom_bucket', 'bloom_lookup', 'bloom_resolve', 'bloom_count', 'part_transpose', 'part_map')):
        big.setdefault(n[:60], []).append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6)
for n, v in big.items():
    print(n, len(v), 'max %.3f ms' % max(v))
PY
