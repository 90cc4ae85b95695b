"""Seeded synthetic genomes, banks and reads (no network, no real assemblies).

Workload of BASELINE.json config 2 / SURVEY.md §8(d): D species genomes of
about 4 Mbp derived from one base genome with 5-20 % per-species substitution
(so cross-species hits are non-trivial), and 150 bp reads drawn uniformly from
them with 1 % substitution errors plus 10 % pure-random reads.  Read sampling
follows the template of ``misclassification_detection/simulate_reads.py:15-55``
(uniform species, uniform start).
"""
from __future__ import annotations

import numpy as np

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def make_genomes(n_species: int, length: int, seed: int = 42, div_min: float = 0.05,
                 div_max: float = 0.20) -> np.ndarray:
    """[n_species, length] uint8 ASCII genomes."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 4, length, dtype=np.uint8)
    out = np.empty((n_species, length), dtype=np.uint8)
    for s in range(n_species):
        div = div_min + (div_max - div_min) * (s / max(1, n_species - 1))
        g = base.copy()
        n_mut = rng.binomial(length, div)
        pos = rng.choice(length, size=n_mut, replace=False) if n_mut < length // 4 else \
            np.flatnonzero(rng.random(length) < div)
        g[pos] = (g[pos] + rng.integers(1, 4, pos.size, dtype=np.uint8)) % 4
        out[s] = ACGT[g]
    return out


def make_reads(genomes: np.ndarray, n_reads: int, read_len: int = 150, seed: int = 42,
               error_rate: float = 0.01, random_frac: float = 0.10) -> tuple[np.ndarray, np.ndarray]:
    """([n_reads, read_len] uint8 ASCII reads, [n_reads] int32 source species or -1)."""
    rng = np.random.default_rng(seed)
    n_sp, glen = genomes.shape
    sp = rng.integers(0, n_sp, n_reads, dtype=np.int64)
    start = rng.integers(0, glen - read_len + 1, n_reads, dtype=np.int64)
    reads = np.empty((n_reads, read_len), dtype=np.uint8)
    chunk = 1 << 18
    cols = np.arange(read_len, dtype=np.int64)
    flat = genomes.reshape(-1)
    for lo in range(0, n_reads, chunk):
        hi = min(n_reads, lo + chunk)
        idx = (sp[lo:hi] * glen + start[lo:hi])[:, None] + cols[None, :]
        reads[lo:hi] = flat[idx]
    # substitution errors
    n_err = rng.binomial(n_reads * read_len, error_rate)
    epos = rng.integers(0, n_reads * read_len, n_err, dtype=np.int64)
    rflat = reads.reshape(-1)
    code = (rflat[epos] >> 1) & 3                   # A0 C1 T2 G3
    newc = (code + rng.integers(1, 4, n_err, dtype=np.uint8)) & 3
    rflat[epos] = np.frombuffer(b"ACTG", dtype=np.uint8)[newc]
    # pure random reads
    n_rand = int(round(n_reads * random_frac))
    ridx = rng.choice(n_reads, size=n_rand, replace=False)
    reads[ridx] = ACGT[rng.integers(0, 4, (n_rand, read_len), dtype=np.uint8)]
    src = sp.astype(np.int32)
    src[ridx] = -1
    return reads, src
