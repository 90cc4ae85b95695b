"""Model-load time (ProbabilisticFilterModel.load reads the
COBS index, 0.5-1 GB, once per `xspect classify` process): config 2's
D=100 species bank (0.61 GB) saved as a COBS classic file, then
Bank.save (3 times) and Bank.open(path) timed with the file in the page cache, best and all of
--reps; the opened bank's image is checked against the saved one.  One
JSON line.
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--path", default="/tmp/xs_open_probe.cobs_classic")
    a = ap.parse_args()
    import torch
    from xspect2_amd._lib import XS_BANK_COBS_CLASSIC
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.synth import make_genomes

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
    path = Path(a.path)
    saves = []
    for _ in range(3):
        t0 = time.perf_counter()
        bank.save(path)
        saves.append((time.perf_counter() - t0) * 1e3)
    want = bank.download()
    bank.close()
    times = []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        b = Bank.open(path, XS_BANK_COBS_CLASSIC, device=0)
        times.append((time.perf_counter() - t0) * 1e3)
        same = bool(np.array_equal(b.download(), want))
        b.close()
        if not same:
            raise SystemExit("opened bank differs from the saved one")
    size = path.stat().st_size
    path.unlink()
    print(json.dumps({"file_bytes": size, "save_ms": saves, "open_ms": times, "best_ms": min(times),
                      "GBps": size / (min(times) * 1e-3) / 1e9, "image_equal": True}), flush=True)


if __name__ == "__main__":
    main()
