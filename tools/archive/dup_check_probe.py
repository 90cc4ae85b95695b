"""Time of PackedIds.has_duplicates (xs_ids_has_duplicates: every file's read
ids are checked when its MatrixResult is made) for 1 M and 12.5 M ids
"read_<i>", best of 3.  Host only.  One JSON line."""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def main():
    from dup_resolve_bench import _ids
    out = {}
    for n in (1_000_000, 12_500_000):
        ids = _ids(0, n)
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            assert not ids.has_duplicates()
            ts.append((time.perf_counter() - t) * 1e3)
        out[f"{n}_ms"] = min(ts)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
