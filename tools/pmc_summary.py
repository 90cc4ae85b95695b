"""Average per-dispatch PMC values of the probe kernel from rocprofv3 CSV passes."""
import collections
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
kern = sys.argv[2] if len(sys.argv) > 2 else "probe_cobs"
agg = collections.defaultdict(list)
dur = []
for f in sorted(root.glob("p*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:45s} n={len(v):3d} avg={sum(v) / len(v):.6g}")
