"""The file -> totals leg of bench.py's end_to_end (config 2: 1M x 150 bp reads
as a FASTQ, device-mode reader, Bank.query_totals per batch), run --reps times
with a 60 ms idle gap between passes, for one

    rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -- python3 tools/e2e_trace.py

run.  The gaps let tools/e2e_trace_table.py cut the trace into passes.  Prints
one JSON line with each pass's host wall time and the batch sizes, and
(--probe-only) the same batches' probes alone, from device-resident copies, so
the table can set the sum of the probes beside the whole pass.
"""
from __future__ import annotations

import argparse
import json
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reads", type=int, default=1_000_000)
    ap.add_argument("--docs", type=int, default=100)
    ap.add_argument("--genome-len", type=int, default=4_000_000)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--gap-ms", type=float, default=60.0)
    args = ap.parse_args()

    import torch
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.file_io import read_batches
    from xspect2_amd.synth import make_genomes, make_reads

    k = 21
    dev = torch.device("cuda", 0)
    genomes = make_genomes(args.docs, args.genome_len, seed=42)
    sig = cobs_signature_size(args.genome_len - k + 1, 7, 0.01)
    bank = Bank.create_cobs(k, 7, [sig], args.docs, [f"sp{i:03d}" for i in range(args.docs)], device=0)
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    go = torch.arange(args.docs + 1, dtype=torch.int64, device=dev) * args.genome_len
    bank.build_device(g, genomes.size, go, args.docs, torch.arange(args.docs, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    del g
    reads, _ = make_reads(genomes, args.reads, 150, seed=42)
    tmp = Path(tempfile.mkdtemp(prefix="xs_e2e_trace_"))
    fq = tmp / "reads.fastq"
    qual = b"I" * 150
    with open(fq, "wb") as fh:
        for lo in range(0, reads.shape[0], 100_000):
            fh.write(b"".join(b"@r%d\n%s\n+\n%s\n" % (i, reads[i].tobytes(), qual)
                              for i in range(lo, min(reads.shape[0], lo + 100_000))))
    out = {"file_bytes": fq.stat().st_size, "reads": int(reads.shape[0]), "passes_ms": [], "batches": None}
    clocks = {"monotonic": time.CLOCK_MONOTONIC, "monotonic_raw": time.CLOCK_MONOTONIC_RAW,
              "boottime": time.CLOCK_BOOTTIME}
    out["pass_clock_ns"] = {c: [] for c in clocks}  # [start, end] of every pass on each host clock
    for _ in range(args.reps):
        time.sleep(args.gap_ms / 1e3)
        c0 = {c: time.clock_gettime_ns(v) for c, v in clocks.items()}
        t = time.perf_counter()
        sizes = []
        for b in read_batches(fq, device=0):
            bank.query_totals(b)
            sizes.append(int(b.n))
        out["passes_ms"].append((time.perf_counter() - t) * 1e3)
        for c, v in clocks.items():
            out["pass_clock_ns"][c].append([c0[c], time.clock_gettime_ns(v)])
        out["batches"] = sizes
    # the same batches' probes alone (device-resident reads, one call per batch), then one 1M call
    time.sleep(args.gap_ms / 1e3)
    s = torch.cuda.current_stream(dev).cuda_stream
    lo = 0
    calls = []
    for n in out["batches"] + [reads.shape[0]]:
        if lo >= reads.shape[0]:
            lo = 0
        part = reads[lo:lo + n]
        d_seqs = torch.from_numpy(part.reshape(-1)).to(dev)
        d_offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * 150
        d_nk = torch.empty(n, dtype=torch.int64, device=dev)
        d_tot = torch.zeros(args.docs + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        bank.query_device(d_seqs, part.size, d_offs, n, 1, None, d_nk, d_tot, stream=s)  # warm
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        bank.query_device(d_seqs, part.size, d_offs, n, 1, None, d_nk, d_tot, stream=s)
        torch.cuda.synchronize(dev)
        calls.append({"reads": int(n), "ms": (time.perf_counter() - t) * 1e3})
        lo += n
    out["probe_alone"] = calls
    print(json.dumps(out), flush=True)
    bank.close()


if __name__ == "__main__":
    main()
