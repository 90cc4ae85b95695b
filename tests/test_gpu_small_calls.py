"""Small host calls (query_small in xs_api.cpp): a request of up to 4096 reads
and 1 MiB of sequence travels in one pinned buffer (host-built unit map, one
H2D copy, the direct probe kernel, one D2H copy, one sync) instead of
query_host's unit pipeline and staging ring (GPU).

Every answer must be the oracle's and the regular path's
(the handle's small_calls option off): hits in every width, k-mer counts, totals, the
per-read best doc; for classic banks of every probe-kernel family, compact
(MLST) banks and rbloom filters, with empty reads, reads shorter than k,
multi-unit reads (> 256 k-mers, counted atomically), non-ACGT bytes and
sampling steps.  Reference: one ``cobs_index.Search.search`` per read
(``probabilistic_filter_model.py:227``) — the call this path serves.
"""
from __future__ import annotations

import numpy as np
import pytest

from test_gpu_parity import _pair, _reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def xs():
    from xspect2_amd import _lib
    from xspect2_amd import bank as bank_mod
    assert _lib.device_count() >= 1, "no HIP device visible"
    return bank_mod


def _best(h: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    m = h.max(axis=1)
    ties = (h == m[:, None]).sum(axis=1)
    best = np.where(ties == 1, h.argmax(axis=1), 0xFFFFFFFF).astype(np.uint32)
    return best, m.astype(np.uint32)


def _requests(rng, seqs, k):
    genome = b"".join(seqs)
    long_read = genome[: max(k + 600, 900)]                      # > 256 k-mers: several units
    base = [b"", b"A" * max(k - 1, 0), b"C" * k, b"G" * (k + 1), long_read]
    reads = _reads(rng, 60, k) + _reads(rng, 20, k, alphabet="ACGTNacgtnRYKM") + \
        [s[: int(rng.integers(k, len(s) + 1))] for s in seqs[:20]] + base
    rng.shuffle(reads)
    return {"one": [seqs[0][:150]], "one_short": [b"ACG"], "few": reads[:7], "many": reads,
            "long_only": [long_read]}


def _check(xs, gb, oracle_query, reqs, steps=(1, 3)):
    cols = gb.num_docs if gb.kind != 2 else 1
    for name, reads in reqs.items():
        for step in steps:
            want_h, want_n = oracle_query(reads, step)
            want_h = np.asarray(want_h, dtype=np.uint32).reshape(len(reads), cols)
            for small in (1, 0):
                gb.set_probe_options(small_calls=small)
                got_h, got_n = gb.query(reads, step=step)
                assert np.array_equal(got_n, want_n) and np.array_equal(got_h, want_h), (name, step, small)
                assert gb.probe_path() == 0
                auto_h, _ = gb.query(reads, step=step, hit_dtype="auto")
                assert auto_h.dtype != np.uint32 or int(want_n.max(initial=0)) > 0xFFFF
                assert np.array_equal(auto_h.astype(np.uint32), want_h), (name, step, small, "auto")
                tot, nk = gb.query_totals(reads, step=step)
                assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
                best, bh, bn, btot = gb.query_best(reads, step=step, want_totals=True)
                wb, wm = _best(want_h)
                assert np.array_equal(best, wb) and np.array_equal(bh, wm) and np.array_equal(bn, want_n)
                assert np.array_equal(btot[:-1], want_h.sum(axis=0, dtype=np.uint64))
                assert int(btot[-1]) == int(want_n.sum())


@pytest.mark.parametrize("D,k,h,sig", [(100, 21, 7, [40_000]), (8, 5, 2, [301]), (200, 21, 7, [12_007]),
                                       (1000, 21, 7, [3_001]), (2100, 21, 7, [4_001]), (129, 31, 1, [20_011])])
def test_small_calls_classic(xs, oracle_mod, D, k, h, sig):
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, seed=D + 3 * k)
    rng = np.random.default_rng(D * 7 + k)
    _check(xs, gb, lambda r, s: ob.query(r, step=s), _requests(rng, seqs, k))
    gb.close()


def test_small_calls_compact(xs, oracle_mod):
    """A compact (MLST-like) bank: 1100 docs in groups of 8 x 64 docs."""
    D, k, page = 1100, 31, 64
    per = 8 * page
    sig = [5_003, 4_001, 3_001]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, 1, sig, page=page, seed=9, per_doc=1)
    assert len(sig) == -(-D // per)
    rng = np.random.default_rng(21)
    _check(xs, gb, lambda r, s: ob.query(r, step=s), _requests(rng, seqs, k), steps=(1,))
    gb.close()


@pytest.mark.parametrize("k", [21, 31])
def test_small_calls_bloom(xs, oracle_mod, k):
    rng = np.random.default_rng(k + 100)
    genome = _reads(rng, 6, k, alphabet="ACGTacgtN", min_len=k, max_len=3000)
    nbytes, K = oracle_mod.BloomFilter.params(sum(len(s) for s in genome) - k + 1, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(genome)
    gb = xs.Bank.create_bloom(k, nbytes, K)
    gb.set_probe_options(bloom_part=0)
    gb.upload(bf.bits)
    _check(xs, gb, lambda r, s: bf.query(r, step=s), _requests(rng, genome, k))
    gb.close()


def test_over_the_limits_take_the_regular_path(xs, oracle_mod):
    """5000 reads (over 4096) and one 2 MiB read (over 1 MiB of sequence):
    the regular path, same answers."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=5)
    rng = np.random.default_rng(6)
    many = _reads(rng, 5000, 21, max_len=160)
    big = [(b"".join(seqs) * 200)[: 2 << 20]]
    for reads in (many, big):
        want_h, want_n = ob.query(reads, step=5)
        got_h, got_n = gb.query(reads, step=5)
        assert np.array_equal(got_h, want_h) and np.array_equal(got_n, want_n)
    gb.close()
