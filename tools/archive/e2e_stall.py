"""Where does the end-to-end device path wait?  (diagnostics, GPU)

The config-2 reads as a FASTQ file -> per-doc totals, three ways, with
timestamps (CLOCK_MONOTONIC ms, the clock of XSPECT2_AMD_FASTX_TRACE):
  seq     FastxReader.next_batch then query_totals, one thread
  gen     file_io.read_batches (batch i+1 parsed on a worker thread while
          batch i is probed), instrumented at every hand-over
  gen_sw  the same with sys.setswitchinterval(1e-4)
"""
from __future__ import annotations

import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))


def ms():
    return time.monotonic() * 1e3


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="seq,gen,gen_sw")
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--reads", type=int, default=1_000_000)
    args = ap.parse_args()
    import torch
    from fx_dev_trace import write_fastq
    from xspect2_amd import file_io
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.synth import make_genomes

    p = Path("/tmp/xs_stall.fastq")
    write_fastq(p, args.reads)
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
    out = {}
    for rep in range(args.reps):
        for mode in args.modes.split(","):
            sys.setswitchinterval(1e-4 if mode == "gen_sw" else 0.005)
            time.sleep(0.3)
            t0 = ms()
            print(f"== {mode} rep {rep} t={t0:.2f}", file=sys.stderr, flush=True)
            if mode == "seq":
                with file_io.FastxReader(p, device=0) as rd:
                    print(f"  opened t={ms():.2f}", file=sys.stderr, flush=True)
                    while True:
                        a = ms()
                        b = rd.next_batch(file_io.DEFAULT_BATCH_TEXT)
                        print(f"  next_batch {a:.2f} -> {ms():.2f} n={b.n}", file=sys.stderr, flush=True)
                        if b.n == 0:
                            break
                        q = ms()
                        bank.query_totals(b)
                        print(f"  query {q:.2f} -> {ms():.2f}", file=sys.stderr, flush=True)
            else:
                for b in file_io.read_batches(p, device=0):
                    q = ms()
                    bank.query_totals(b)
                    print(f"  got batch n={b.n}; query {q:.2f} -> {ms():.2f}", file=sys.stderr, flush=True)
            dt = ms() - t0
            out.setdefault(mode, []).append(round(dt, 2))
            print(f"== {mode} {dt:.2f} ms", file=sys.stderr, flush=True)
    sys.setswitchinterval(0.005)
    print(json.dumps(out))


if __name__ == "__main__":
    os.environ.setdefault("XSPECT2_AMD_FASTX_TRACE", "1")
    main()
