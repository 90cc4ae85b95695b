"""Device-mode reader timing on one file (diagnostics, GPU): the host reader
and the device reader over the same FASTQ, --reps passes each, with
XSPECT2_AMD_FASTX_TRACE per-window phase lines on stderr."""
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


def write_fastq(path: Path, n: int, L: int = 150, seed: int = 42) -> None:
    rng = np.random.default_rng(seed)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    with open(path, "wb") as fh:
        for c0 in range(0, n, 100_000):
            m = min(100_000, n - c0)
            seqs = acgt[rng.integers(0, 4, (m, L))]
            fh.write(b"".join(b"@read_%d\n%s\n+\n%s\n" % (c0 + i, seqs[i].tobytes(), b"I" * L) for i in range(m)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--batch-mb", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--bank", action="store_true", help="also time file -> hits / totals (config-2 bank)")
    args = ap.parse_args()
    os.environ.setdefault("XSPECT2_AMD_FASTX_TRACE", "1")
    from xspect2_amd.file_io import read_batches
    p = Path("/tmp/xs_trace.fastq")
    write_fastq(p, args.reads)
    size = p.stat().st_size
    res = {"file_bytes": size, "reads": args.reads, "batch_mb": args.batch_mb}
    mb = args.batch_mb << 20
    for name, kw in (("host", {}), ("device", {"device": 0})):
        ts = []
        for _ in range(args.reps):
            time.sleep(0.3)
            t = time.perf_counter()
            n = sum(b.n for b in read_batches(p, mb, threads=args.threads, **kw))
            ts.append(time.perf_counter() - t)
            assert n == args.reads
            print(f"{name} pass {ts[-1] * 1e3:.1f} ms", file=sys.stderr, flush=True)
        res[f"{name}_ms"] = [round(x * 1e3, 2) for x in ts]
        res[f"{name}_GBps_best"] = size / min(ts) / 1e9
    if args.bank:
        import torch
        from xspect2_amd.bank import Bank, cobs_signature_size
        from xspect2_amd.synth import make_genomes
        k, D, G = 21, 100, 4_000_000
        dev = torch.device("cuda", 0)
        genomes = make_genomes(D, G, seed=42)
        bank = Bank.create_cobs(k, 7, [cobs_signature_size(G - k + 1, 7, 0.01)], D, [f"sp{i}" for i in range(D)])
        g = torch.from_numpy(genomes.reshape(-1)).to(dev)
        go = torch.arange(D + 1, dtype=torch.int64, device=dev) * G
        bank.build_device(g, genomes.size, go, D, torch.arange(D, dtype=torch.int32, device=dev),
                          stream=torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        del g
        legs = {"hits": lambda b: bank.query(b, hit_dtype="auto"), "totals": lambda b: bank.query_totals(b)}
        for rep in range(args.reps):
            for name in (["hits", "totals"] if rep % 2 == 0 else ["totals", "hits"]):
                for mode, kw in (("device", {"device": 0}), ("host", {})):
                    time.sleep(0.3)  # the box's CPU share (cgroup quota) refills between legs
                    t = time.perf_counter()
                    if mode == "device":
                        print(f"  leg {name} t={time.monotonic() * 1e3:.2f}", file=sys.stderr, flush=True)
                    for b in read_batches(p, mb, **kw):
                        q0 = time.monotonic() * 1e3
                        legs[name](b if mode == "device" else b.packed)
                        if mode == "device":
                            print(f"  query t={q0:.2f} n={b.n} {time.monotonic() * 1e3 - q0:.2f} ms",
                                  file=sys.stderr, flush=True)
                    dt = time.perf_counter() - t
                    res.setdefault(f"e2e_{mode}_{name}_ms", []).append(round(dt * 1e3, 2))
                    print(f"e2e {mode} {name} {dt * 1e3:.1f} ms", file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
