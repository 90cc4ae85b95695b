"""Hit matrices back to host memory (xs_query / xs_query_hits, GPU).

The rows of every chunk of a host call go back on a worker thread while the
next chunks are probed (HitSink, xs_api.cpp): narrowed on the device to the
narrowest width that holds the batch's largest k-mer count, staged through a
ring of three 32 MiB pinned slots and widened on the host into the caller's
array; a pinned destination takes the rows by DMA in its own width.  Every
combination must give the oracle's matrix: uint32 into the pooled pageable
array Bank.query returns by default, into a fresh np.empty and into a pinned
array; uint8 / uint16 outputs; wire widths 1 (150 bp reads), 2 (reads of
> 255 k-mers) and 4 (reads of > 65535 k-mers); batches of several host
chunks and several 32 MiB pieces (the ring wraps).  Reference: the per-read
``cobs_index.Search.search`` (probabilistic_filter_model.py:227) that
xs_query batches.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import _pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def xs():
    from xspect2_amd import _lib
    from xspect2_amd import bank as bank_mod
    assert _lib.device_count() >= 1, "no HIP device visible"
    return bank_mod


def _windows(rng, seqs, n, lo, hi):
    genome = b"".join(seqs)
    out = []
    for _ in range(n):
        L = int(rng.integers(lo, hi + 1))
        o = int(rng.integers(0, len(genome) - L))
        out.append(genome[o:o + L])
    return out


def _all_outputs_equal_oracle(xs, gb, ob, reads):
    from xspect2_amd.packing import pack_sequences
    pr = pack_sequences(reads)
    want_h, want_n = ob.query_packed(pr.buf, pr.offsets, threads=0)
    D = gb.num_docs
    got, nk = gb.query(pr)                                          # pooled pageable uint32
    assert got.dtype == np.uint32 and np.array_equal(nk, want_n)
    assert np.array_equal(got, want_h)
    fresh = np.empty((pr.n, D), np.uint32)                         # never touched
    gb.query(pr, out=fresh)
    assert np.array_equal(fresh, want_h)
    pinned = xs.pinned_empty((pr.n, D), np.uint32)                 # DMA straight in
    gb.query(pr, out=pinned)
    assert np.array_equal(pinned, want_h)
    top = int(want_h.max()) if want_h.size else 0
    for dt in (np.uint8, np.uint16):
        if top <= np.iinfo(dt).max and int(want_n.max()) <= np.iinfo(dt).max:
            h, _ = gb.query(pr, hit_dtype=dt)
            assert h.dtype == dt and np.array_equal(h.astype(np.uint32), want_h)
    return want_h


def test_u32_matrix_many_chunks_and_pieces(xs, oracle_mod):
    """600 k reads of 150 bp (90 MB of sequence: four host chunks; a 60 MB
    uint8 wire, two 32 MiB pieces; 240 MB of uint32 rows)."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=21)
    rng = np.random.default_rng(21)
    reads = _windows(rng, seqs, 600_000, 150, 150)
    want = _all_outputs_equal_oracle(xs, gb, ob, reads)
    assert int(want.sum()) > 0
    gb.close()


def test_u16_wire_long_reads(xs, oracle_mod):
    """Reads of 300-2000 bp (up to 1980 k-mers: the rows cross as uint16 and
    are widened to uint32) mixed with short and empty reads."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=22)
    rng = np.random.default_rng(22)
    reads = _windows(rng, seqs, 40_000, 300, 2000) + [b"", b"ACGT", seqs[0][:21]]
    rng.shuffle(reads)
    want = _all_outputs_equal_oracle(xs, gb, ob, reads)
    assert int(want.max()) > 255
    gb.close()


def test_u32_wire_very_long_reads(xs, oracle_mod):
    """Three reads of 70 kbp (> 65535 k-mers each: the rows cross as uint32)
    among 150 bp reads."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=23, per_doc=40)
    rng = np.random.default_rng(23)
    genome = b"".join(seqs)
    assert len(genome) > 80_000
    reads = _windows(rng, seqs, 2000, 150, 150) + [genome[i * 5000:i * 5000 + 70_000] for i in range(3)]
    want = _all_outputs_equal_oracle(xs, gb, ob, reads)
    assert int(want.max()) > 65535
    gb.close()


def test_pinned_buffers_are_given_back(xs):
    """xs_host_alloc / xs_host_free over both kinds of pinned memory (2 MiB
    and more: registered huge-page mappings; less: hipHostMalloc), 24
    rounds of 256 MiB + 1 MiB: the process's resident memory does not grow
    by more than a round's worth (a mapping kept after its free would add
    256 MiB a round), and each buffer holds what was written to it."""
    import gc

    def rss_mb():
        for line in open("/proc/self/status"):
            if line.startswith("VmRSS:"):
                return int(line.split()[1]) / 1024
        return 0.0

    base = None
    for i in range(24):
        big = xs.pinned_empty((256 << 20,), np.uint8)
        small = xs.pinned_empty((1 << 20,), np.uint8)
        big[:: 1 << 20] = i
        small[:] = i
        assert int(big[(255 << 20)]) == i and int(small[-1]) == i
        del big, small
        gc.collect()
        if i == 3:
            base = rss_mb()
    assert rss_mb() - base < 400, (base, rss_mb())


def test_large_host_batch_argument_errors(xs, oracle_mod):
    """The per-read passes of a host batch run on several threads from 2^18
    reads on: a decreasing offset anywhere is refused, and a read too long
    for a narrow output is reported by its index (the first such read)."""
    from xspect2_amd import _lib
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=31)
    n = 300_000
    seq = (b"ACGT" * 15) * n  # 300 k reads of 60 bp
    offs = np.arange(n + 1, dtype=np.uint64) * 60
    bad = offs.copy()
    bad[250_001] = bad[250_000] - 1  # in the last threads' ranges
    hits = np.empty((n, 100), np.uint32)
    nk = np.empty(n, np.uint64)
    lib = _lib.load()
    rc = lib.xs_query(gb.handle, seq, bad.ctypes.data, n, 1, hits.ctypes.data, nk.ctypes.data)
    assert rc == _lib.XS_ERR_ARG and b"non-decreasing" in lib.xs_last_error()
    # reads 200000 and 280000 have 280 k-mers: too many for uint8 counts; the first is named
    lens = np.full(n, 60, dtype=np.uint64)
    lens[200_000] = lens[280_000] = 300
    offs2 = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs2[1:])
    seq2 = (b"ACGT" * 75) * 2 + seq[: int(offs2[-1]) - 600]
    out8 = np.empty((n, 100), np.uint8)
    rc = lib.xs_query_hits(gb.handle, seq2, offs2.ctypes.data, n, 1, out8.ctypes.data, 1, nk.ctypes.data)
    assert rc == _lib.XS_ERR_ARG and b"read 200000 has 280 sampled k-mers" in lib.xs_last_error()
    # and a valid large batch still equals the oracle
    got, got_nk = gb.query([seq[:60]] * 10 + [seqs[0][:150]])
    want, want_nk = ob.query([seq[:60]] * 10 + [seqs[0][:150]])
    assert np.array_equal(got, want) and np.array_equal(got_nk, want_nk)
    gb.close()
