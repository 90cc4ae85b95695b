"""Where a fresh pageable output's first-touch time goes in xs_query (config
2's 1M x 100 uint32 matrix), on the box: Bank.query into the host pool
(pages faulted once), into a fresh np.empty array, and into a fresh array
pre-faulted by 8 threads first (its memset timed apart); with the process's
AnonHugePages before and after each fresh call (/proc/self/smaps_rollup), to
see whether the faults took 2 MiB pages.  One JSON line.
"""
from __future__ import annotations

import ctypes
import json
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
libc = ctypes.CDLL(None)
libc.memset.restype = ctypes.c_void_p
libc.memset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]


def anon_huge_kb() -> int:
    for line in Path("/proc/self/smaps_rollup").read_text().splitlines():
        if line.startswith("AnonHugePages:"):
            return int(line.split()[1])
    return -1


def touch8(a: np.ndarray) -> float:
    n, p = a.nbytes, a.ctypes.data
    per = (n + 7) // 8
    t0 = time.perf_counter()
    th = [threading.Thread(target=libc.memset, args=(p + i * per, 0, min(per, n - i * per))) for i in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return (time.perf_counter() - t0) * 1e3


def main():
    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.packing import pack_fixed
    from xspect2_amd.synth import make_genomes, make_reads

    D, L, k = 100, 4_000_000, 21
    dev = torch.device("cuda", 0)
    genomes = make_genomes(D, L, seed=42)
    sig = cobs_signature_size(L - k + 1, 7, 0.01)
    bank = Bank.create_cobs(k, 7, [sig], D, [f"sp{i}" for i in range(D)], device=0)
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(D + 1, dtype=torch.int64, device=dev) * L
    bank.build_device(g, genomes.size, go, D, torch.arange(D, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    reads, _ = make_reads(genomes, 1_000_000, 150, seed=42)
    pr = pack_fixed(reads)
    shape = (pr.n, D)

    def timed(fn):
        t0 = time.perf_counter()
        fn()
        return (time.perf_counter() - t0) * 1e3

    bank.query(pr)  # warm
    out = {"pooled_ms": min(timed(lambda: bank.query(pr)) for _ in range(3))}
    fresh, huge = [], []
    for _ in range(3):
        a = np.empty(shape, np.uint32)
        h0 = anon_huge_kb()
        fresh.append(timed(lambda: bank.query(pr, out=a)))
        huge.append(anon_huge_kb() - h0)
        del a
    out["fresh_ms"], out["fresh_anon_huge_kb"] = min(fresh), huge
    cyc, frees = [], []
    for _ in range(3):  # as bench.py's leg: allocate, query, drop (the unmap inside the time)
        t0 = time.perf_counter()
        a = np.empty(shape, np.uint32)
        bank.query(pr, out=a)
        t1 = time.perf_counter()
        del a
        t2 = time.perf_counter()
        cyc.append((t2 - t0) * 1e3)
        frees.append((t2 - t1) * 1e3)
    out["fresh_cycle_ms"], out["free_ms"] = cyc, frees
    pre, q = [], []
    for _ in range(3):
        a = np.empty(shape, np.uint32)
        pre.append(touch8(a))
        q.append(timed(lambda: bank.query(pr, out=a)))
        del a
    out["pretouch8_ms"], out["after_pretouch8_query_ms"] = min(pre), min(q)
    a = np.empty(shape, np.uint32)
    h0 = anon_huge_kb()
    out["touch8_alone_ms"] = touch8(a)
    out["touch8_anon_huge_kb"] = anon_huge_kb() - h0
    t0 = time.perf_counter()
    del a
    out["free_after_touch8_ms"] = (time.perf_counter() - t0) * 1e3
    a = np.empty(shape, np.uint32)
    t0 = time.perf_counter()
    libc.memset(a.ctypes.data, 0, a.nbytes)
    out["touch1_ms"] = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    del a
    out["free_after_touch1_ms"] = (time.perf_counter() - t0) * 1e3
    print(json.dumps(out), flush=True)
    bank.close()


if __name__ == "__main__":
    main()
