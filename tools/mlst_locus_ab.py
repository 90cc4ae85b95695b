"""Time one MLST locus probe per locus size (diagnostic).

A locus of N alleles (mutated copies of one 620-bp sequence, 400-600 bp each,
bench.py's generator) in a compact bank of 64-byte pages (512 alleles per
group, so N <= 512 / 1024 / 1536 / 2048 gives 1-4 groups), k = 31, one hash,
fpr 0.001.  1 M x 150 bp reads: one in seven from this locus's alleles, the
rest random sequence (WGS-like input), or with --foreign loci from six other
loci's alleles as in bench.py's config 4 (few distinct k-mers: their rows stay
in L2).  The library's query_device writes the n x N u32 hit matrix, as in
bench.py's MLST step; times are HIP events around 10 calls after 3 warm-up
calls.  Prints one JSON line per locus size.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from xspect2_amd.bank import Bank, cobs_signature_size  # noqa: E402


def make_alleles(rng, n_alleles):
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    base = acgt[rng.integers(0, 4, 620)]
    alleles = []
    for _ in range(n_alleles):
        L = int(rng.integers(400, 601))
        a = base[:L].copy()
        pos = rng.integers(0, L, int(rng.integers(0, 12)))
        a[pos] = acgt[(np.searchsorted(acgt, a[pos]) + 1) % 4]
        alleles.append(a)
    return alleles


def read_from(rng, alleles):
    a = alleles[int(rng.integers(0, len(alleles)))]
    st = int(rng.integers(0, a.size - 150 + 1))
    return a[st:st + 150]


def locus(n_alleles: int, n_reads: int, k: int, dev, s, foreign: str):
    rng = np.random.default_rng(4242 + n_alleles)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    alleles = make_alleles(rng, n_alleles)
    alleles.sort(key=lambda a: a.size)
    per = 8 * 64
    sig = [cobs_signature_size(max(a.size for a in alleles[g:g + per]) - k + 1, 1, 0.001)
           for g in range(0, n_alleles, per)]
    bank = Bank.create_cobs(k, 1, sig, n_alleles, [f"Allele_ID_{i}" for i in range(n_alleles)],
                            page_size=64, compact=True, device=dev.index)
    buf = np.concatenate(alleles)
    offs = np.zeros(n_alleles + 1, dtype=np.int64)
    offs[1:] = np.cumsum([a.size for a in alleles])
    bank.build_device(torch.from_numpy(buf).to(dev), buf.size, torch.from_numpy(offs).to(dev), n_alleles,
                      torch.arange(n_alleles, dtype=torch.int32, device=dev), stream=s)
    reads = acgt[rng.integers(0, 4, (n_reads, 150))]
    others = [make_alleles(rng, 1430) for _ in range(6)] if foreign == "loci" else None
    own = rng.random(n_reads) < 1 / 7
    for i in range(n_reads):
        if own[i]:
            reads[i] = read_from(rng, alleles)
        elif others is not None:
            reads[i] = read_from(rng, others[i % 6])
    return bank, len(sig), reads


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = torch.cuda.Stream(dev)
    n, k = 1_000_000, 31
    args = sys.argv[1:]
    foreign = "random"
    if args[:2] == ["--foreign", "loci"] or args[:2] == ["--foreign", "random"]:
        foreign, args = args[1], args[2:]
    for n_alleles in [int(x) for x in (args or ["400", "900", "1430", "2000"])]:
        bank, groups, reads = locus(n_alleles, n, k, dev, st.cuda_stream, foreign)
        d_seqs = torch.from_numpy(reads.reshape(-1)).to(dev)
        d_offs = torch.arange(0, (n + 1) * 150, 150, dtype=torch.int64, device=dev)
        d_hits = torch.empty((n, n_alleles), dtype=torch.int32, device=dev)
        d_nk = torch.empty(n, dtype=torch.int64, device=dev)
        d_tot = torch.empty(n_alleles + 1, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)

        def call():
            bank.query_device(d_seqs, d_seqs.numel(), d_offs, n, 1, d_hits, d_nk, d_tot, stream=st.cuda_stream)

        for _ in range(3):
            call()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            call()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 10
        kmers = n * (150 - k + 1)
        print(json.dumps({"alleles": n_alleles, "groups": groups, "foreign": foreign, "ms_per_call": round(ms, 4),
                          "probes_per_s": kmers * n_alleles / (ms * 1e-3),
                          "hits_checksum": int(d_hits.sum().item()), "kmers": int(d_nk.sum().item())}), flush=True)
        bank.close()


if __name__ == "__main__":
    main()
