"""First-touch cost of a fresh 400 MB pageable array (config 2's uint32 hit
matrix) on this host, with and without transparent huge pages, written by 1
or 8 threads (the faults of 4 KiB pages neither batch nor spread
over threads).  Each case: a fresh anonymous mapping, optionally
madvise(MADV_HUGEPAGE), then memset by T threads (ctypes releases the GIL);
the second memset of the same mapping is the write alone.  Prints one JSON
line with the host's THP settings and every case's best-of-3 times.

    python tools/thp_probe.py [--mb 400]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import mmap
import threading
import time
from pathlib import Path

libc = ctypes.CDLL(None, use_errno=True)
libc.memset.restype = ctypes.c_void_p
libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE = 14


def _fill(addr: int, n: int, threads: int) -> float:
    per = (n + threads - 1) // threads
    per = (per + (2 << 20) - 1) // (2 << 20) * (2 << 20)  # whole 2 MiB pieces per thread
    t0 = time.perf_counter()
    th = [threading.Thread(target=libc.memset, args=(addr + i * per, 1, min(per, n - i * per)))
          for i in range(threads) if i * per < n]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return (time.perf_counter() - t0) * 1e3


def case(nbytes: int, huge: bool, threads: int) -> dict:
    firsts, seconds = [], []
    for _ in range(3):
        m = mmap.mmap(-1, nbytes + (2 << 20), flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        base = ctypes.addressof(ctypes.c_char.from_buffer(m))
        addr = (base + (2 << 20) - 1) // (2 << 20) * (2 << 20)  # 2 MiB aligned
        if huge:
            rc = libc.madvise(addr, nbytes, MADV_HUGEPAGE)
            if rc != 0:
                return {"error": f"madvise errno {ctypes.get_errno()}"}
        firsts.append(_fill(addr, nbytes, threads))
        seconds.append(_fill(addr, nbytes, threads))
        del base
        m.close()
    return {"first_touch_ms": min(firsts), "rewrite_ms": min(seconds)}


def case_numpy(nbytes: int, threads: int) -> dict:
    """The same on an np.empty array (glibc's mmap'd chunk: page aligned plus a
    16-byte header), advised from its first whole page, as HitSink does."""
    import numpy as np
    firsts, seconds = [], []
    for _ in range(3):
        arr = np.empty(nbytes, np.uint8)
        p = arr.ctypes.data
        a = (p + 4095) & ~4095
        e = (p + nbytes) & ~4095
        rc = libc.madvise(a, e - a, MADV_HUGEPAGE)
        if rc != 0:
            return {"error": f"madvise errno {ctypes.get_errno()}"}
        firsts.append(_fill(p, nbytes, threads))
        seconds.append(_fill(p, nbytes, threads))
        del arr
    return {"first_touch_ms": min(firsts), "rewrite_ms": min(seconds), "addr_mod_2MiB": p % (2 << 20)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=400)
    a = ap.parse_args()
    n = a.mb << 20
    thp = {}
    for f in ("enabled", "defrag"):
        p = Path("/sys/kernel/mm/transparent_hugepage") / f
        thp[f] = p.read_text().strip() if p.exists() else None
    out = {"bytes": n, "thp": thp}
    for huge in (False, True):
        for t in (1, 8):
            out[f"{'huge' if huge else 'plain'}_t{t}"] = case(n, huge, t)
    out["numpy_huge_t8"] = case_numpy(n, 8)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
