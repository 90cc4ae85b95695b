# Round 4: kernel trace of the end-to-end device path (reader + probe), to
# split the reader's phases into kernel time and gaps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04e; mkdir -p $F
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$F/trace" -o run -- python3 "$GRAFT_REPO_ROOT/tools/e2e_seq.py" --reps 5 > "$GRAFT_REPO_ROOT/$F/seq.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$F/seq.log"; exit 15; }
cd "$GRAFT_REPO_ROOT" && grep "rep " $F/seq.log
f=$(find $F/trace -name "*kernel_stats.csv" | head -1); cp $f $F/kernel_stats.csv; head -40 $F/kernel_stats.csv | cut -d, -f1-8
t=$(find $F/trace -name "*kernel_trace.csv" | head -1); python3 - "$t" > $F/timeline.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 400 dispatches: the last rep's kernels in order, with gaps
last = rows[-400:]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
    print(f"{(s - t0) / 1e3:9.1f} us  dur {(e - s) / 1e3:8.1f}  gap {(s - prev_end) / 1e3:8.1f}  {name}")
    prev_end = max(prev_end, e)
PY
rm -f $t
tail -120 $F/timeline.txt
