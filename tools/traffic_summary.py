"""Per-dispatch probe-kernel traffic from tools/gpu/gpu_pmc_traffic.sh's rocprofv3 passes.

hbm_bytes_per_launch = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): FETCH_SIZE
counts 128-B requests at 64 B on gfx950 (MI355X_MICROARCH.md, HBM section).
Memory-side counters include Infinity-Cache hits.
"""
import collections
import csv
import json
import sys
from pathlib import Path

root = Path(sys.argv[1])
out = {}
for wdir in sorted(p for p in root.iterdir() if p.is_dir()):
    agg = collections.defaultdict(list)
    kname = None
    for f in wdir.glob("*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "probe_" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
                kname = r["Kernel_Name"]
    avg = {k: sum(v) / len(v) for k, v in agg.items()}
    bench = json.loads((root / f"{wdir.name}.f.json").read_text().strip().splitlines()[-1])
    entry = {"workload": wdir.name, "reads": bench["config"]["reads_per_gpu"], "kernel": kname,
             "dispatches": len(agg.get("FETCH_SIZE", [])), **{k: v for k, v in avg.items()}}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        entry["hbm_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
    if "TCC_EA0_RDREQ_128B_sum" in avg:
        entry["read_bytes_from_requests"] = (avg["TCC_EA0_RDREQ_128B_sum"] * 128 + avg.get("TCC_EA0_RDREQ_64B_sum", 0) * 64
                                             + avg.get("TCC_EA0_RDREQ_32B_sum", 0) * 32)
    out[wdir.name] = entry
out["source"] = ("rocprofv3 --pmc, separate FETCH_SIZE / WRITE_SIZE / TCC_EA0_RDREQ* passes over "
                 "bench.py --steps 3 --warmup 1; per-dispatch average of the probe kernel; "
                 "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KB (gfx950 FETCH_SIZE correction)")
print(json.dumps(out, indent=1))
