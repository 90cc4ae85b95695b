"""Result-save time (`xspect classify` writes ModelResult.save's
JSON, result.py:151-202): a MatrixResult of --reads reads x 100 docs with
uint8 counts of a config-2-like spread (most docs 0-5, one doc near the
read's k-mer count), ids "read_<i>", saved --reps times into --dir; best and
all times, the JSON size and its rate.  Host only.  One JSON line.

    python tools/save_probe.py [--reads 1000000] [--dir /tmp]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--dir", default="/tmp")
    ap.add_argument("--null", action="store_true", help="also save into /dev/null: the formatting alone")
    a = ap.parse_args()
    from xspect2_amd.packing import PackedIds
    from xspect2_amd.result import MatrixResult
    sys.path.insert(0, str(ROOT / "tools"))
    from dup_resolve_bench import _ids

    n, D = a.reads, 100
    rng = np.random.default_rng(5)
    hits = rng.integers(0, 6, (n, D), dtype=np.uint8)
    hits[np.arange(n), rng.integers(0, D, n)] = rng.integers(100, 131, n, dtype=np.uint8)
    nk = np.full(n, 130, dtype=np.uint64)
    ids = _ids(0, n)
    assert isinstance(ids, PackedIds)
    res = MatrixResult("acinetobacter-species", ids, [f"GCF_{i:09d}" for i in range(D)], hits, nk)
    res.input_source = "reads.fq"
    path = Path(a.dir) / "xs_save_probe.json"
    times = []
    for _ in range(a.reps):
        if path.exists():
            path.unlink()
        t0 = time.perf_counter()
        res.save(path)
        times.append(time.perf_counter() - t0)
    size = path.stat().st_size
    path.unlink()
    out = {"reads": n, "docs": D, "json_bytes": size, "save_s": times, "best_s": min(times),
           "GBps": size / min(times) / 1e9, "cpus": os.cpu_count()}
    if a.null:  # the same save with every write discarded
        null = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            res.save(Path("/dev/null"))
            null.append(time.perf_counter() - t0)
        out["devnull_s"] = null
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
