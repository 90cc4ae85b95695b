"""Fixed cost of one probe call vs its size (diagnostics, GPU): config-2
bank, device-resident reads; for each batch size, the probe's HIP-event time
and per-pass times (xs_bank_pass_stats), and the wall time of the device-batch
host call (xs_query_hits_device with totals, as a reader batch is probed)."""
from __future__ import annotations

import ctypes
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    import torch
    from xspect2_amd import _lib
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.synth import make_genomes, make_reads

    k, D, G = 21, 100, 4_000_000
    dev = torch.device("cuda", 0)
    genomes = make_genomes(D, G, seed=42)
    bank = Bank.create_cobs(k, 7, [cobs_signature_size(G - k + 1, 7, 0.01)], D, [f"sp{i}" for i in range(D)])
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(D + 1, dtype=torch.int64, device=dev) * G
    s = torch.cuda.current_stream(dev)
    bank.build_device(g, genomes.size, go, D, torch.arange(D, dtype=torch.int32, device=dev), stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    reads, _ = make_reads(genomes, 1_000_000, 150, seed=42)
    d_seq = torch.from_numpy(reads.reshape(-1)).to(dev)
    lib = _lib.load()
    out = {}
    for n in (26_000, 53_000, 106_000, 212_000, 423_000, 1_000_000):
        d_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * 150
        tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
        for _ in range(3):
            bank.query_device(d_seq, n * 150, d_off, n, 1, None, None, tot, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        bank.set_profiling(True)
        bank.probe_stats()
        bank.pass_stats()
        reps = 10
        for _ in range(reps):
            bank.query_device(d_seq, n * 150, d_off, n, 1, None, None, tot, stream=s.cuda_stream)
        torch.cuda.synchronize(dev)
        launches, ms_tot, _ = bank.probe_stats()
        passes = {k2: round(v[0] / max(1, launches), 4) for k2, v in bank.pass_stats().items()}
        bank.set_profiling(False)
        # the host call a reader batch takes (totals back to the host)
        th = np.zeros(D + 1, dtype=np.uint64)
        walls = []
        for _ in range(reps):
            t = time.perf_counter()
            rc = lib.xs_query_hits_device(bank.handle, d_seq.data_ptr(), n * 150, d_off.data_ptr(), n, 150, 1,
                                          None, 4, None, th.ctypes.data)
            walls.append((time.perf_counter() - t) * 1e3)
            assert rc == 0
        out[n] = {"probe_ms": round(ms_tot / launches, 4), "passes_ms": passes,
                  "host_call_ms_median": round(float(np.median(walls)), 4), "path": bank.probe_path()}
        print(n, json.dumps(out[n]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
