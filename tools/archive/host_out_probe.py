"""Where the time of xs_query's host hit matrix goes (bench.py host_path):
config 2's 1M x 150 bp reads from pageable host memory against the D=100
species bank, best of --reps calls each:

  u32_pooled     Bank.query's default: xs_query's uint32 matrix into a pageable array from the
                 recycled host pool (bench's hits_u32_pageable)
  u32_fresh      the same into a never-touched np.empty array (bench's hits_u32_fresh_pageable)
  u32_touched    the same into one reused (already faulted) pageable array
  u8_fresh       xs_query_hits uint8 into a fresh pageable array
  u8_pinned      xs_query_hits uint8 into a reused pinned array (bench's hits)
  totals         xs_query_totals (no matrix)
  touch_400MB    np.empty of the u32 matrix's size + one write per 4 KiB page (first-touch cost alone)
Prints one JSON line.
"""
from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size, pinned_empty
    from xspect2_amd.packing import pack_fixed
    from xspect2_amd.synth import make_genomes, make_reads

    reps = 5
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
    touched = np.zeros((pr.n, D), np.uint32)
    pin8 = pinned_empty((pr.n, D), np.uint8)

    def best(fn):
        fn()
        ts = []
        for _ in range(reps):
            t = time.perf_counter()
            fn()
            ts.append((time.perf_counter() - t) * 1e3)
        return {"best_ms": min(ts), "median_ms": sorted(ts)[len(ts) // 2]}

    def touch():
        a = np.empty((pr.n, D), np.uint32)
        a.reshape(-1).view(np.uint8)[::4096] = 0

    out = {
        "u32_pooled": best(lambda: bank.query(pr)),
        "u32_fresh": best(lambda: bank.query(pr, out=np.empty((pr.n, D), np.uint32))),
        "u32_touched": best(lambda: bank.query(pr, out=touched)),
        "u8_fresh": best(lambda: bank.query(pr, hit_dtype=np.uint8)),
        "u8_pinned": best(lambda: bank.query(pr, hit_dtype=np.uint8, out=pin8)),
        "totals": best(lambda: bank.query_totals(pr)),
        "touch_400MB": best(touch),
    }
    h, _ = bank.query(pr)
    h8, _ = bank.query(pr, hit_dtype=np.uint8)
    out["u32_equals_u8"] = bool(np.array_equal(h, h8.astype(np.uint32)))
    print(json.dumps(out), flush=True)
    bank.close()


if __name__ == "__main__":
    main()
