"""Per-kernel PMC averages from rocprofv3 --pmc passes (one sub-directory per pass).

usage: pmc_kernels.py <dir> <label> [out.json]
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) KB per dispatch: FETCH_SIZE counts
128-B requests at 64 B on gfx950 (MI355X_MICROARCH.md, HBM section); the
memory-side counters include Infinity-Cache hits.
"""
import collections
import csv
import json
import sys
from pathlib import Path

root = Path(sys.argv[1])
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in list(root.glob("*/run_counter_collection.csv")) + list(root.glob("*/*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        if "build_" in name:
            continue
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {}
for k, c in agg.items():
    e = {n: sum(v) / len(v) for n, v in c.items()}
    e["dispatches"] = max(len(v) for v in c.values())
    if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
        e["hbm_bytes"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
    if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e and e["TCC_HIT_sum"] + e["TCC_MISS_sum"]:
        e["l2_hit_rate"] = e["TCC_HIT_sum"] / (e["TCC_HIT_sum"] + e["TCC_MISS_sum"])
    per[k] = e
out = {"label": sys.argv[2], "kernels": per,
       "hbm_bytes_per_step": sum(v.get("hbm_bytes", 0) for v in per.values()),
       "source": "rocprofv3 --pmc passes (FETCH_SIZE; WRITE_SIZE; TCC_HIT_sum TCC_MISS_sum), per-dispatch averages"}
print(json.dumps(out, indent=1))
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
