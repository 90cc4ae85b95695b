"""Small-call latency of the host API (a serving loop's shape: one request =
one C-ABI call on a resident bank).  Config-2 bank (D=100, 0.61 GB), reads
from its genomes; for each batch size, the median wall time of
Bank.query(hit_dtype="auto") (H2D, probe, D2H of the narrowed hit matrix),
Bank.query_totals and the per-read best doc, over --reps calls after warmup.
Prints one JSON line."""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1,10,100,1000,10000,100000")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--docs", type=int, default=100)
    ap.add_argument("--genome-len", type=int, default=4_000_000)
    args = ap.parse_args()

    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.packing import pack_fixed
    from xspect2_amd.synth import make_genomes, make_reads

    dev = torch.device("cuda", 0)
    k = 21
    genomes = make_genomes(args.docs, args.genome_len, seed=42)
    bank = Bank.create_cobs(k, 7, [cobs_signature_size(args.genome_len - k + 1, 7, 0.01)], args.docs,
                            [f"sp{i:03d}" for i in range(args.docs)], device=0)
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(args.docs + 1, dtype=torch.int64, device=dev) * args.genome_len
    bank.build_device(g, genomes.size, go, args.docs, torch.arange(args.docs, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    sizes = [int(s) for s in args.sizes.split(",")]
    reads, _ = make_reads(genomes, max(sizes), 150, seed=7)
    out = {"docs": args.docs, "bank_bytes": int(bank.info.device_bytes), "reps": args.reps, "sizes": {}}
    for n in sizes:
        pr = pack_fixed(reads[:n])
        row = {}
        for name, fn in (("hits", lambda: bank.query(pr, hit_dtype="auto")),
                         ("totals", lambda: bank.query_totals(pr)),
                         ("best", lambda: bank.query_best(pr))):
            for _ in range(3):
                fn()
            reps = args.reps if n <= 10_000 else max(5, args.reps // 10)
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            row[name] = {"median_us": float(np.median(ts) * 1e6), "p90_us": float(np.percentile(ts, 90) * 1e6)}
        row["probe_path"] = int(bank.probe_path()) if hasattr(bank, "probe_path") else None
        out["sizes"][str(n)] = row
        print(n, json.dumps(row), file=sys.stderr, flush=True)
    bank.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
