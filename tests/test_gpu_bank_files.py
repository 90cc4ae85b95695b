"""Bank files onto the device (xs_bank_open / xs_bank_open_docs, GPU).

A model load reads the whole index (ProbabilisticFilterModel.load,
probabilistic_filter_model.py:351-391); the library streams the payload in
32 MiB pieces through a ring of three pinned slots.  These cases make the
ring wrap several times, with a last piece that is not a whole piece and
rows (13 B for 100 docs) that straddle the pieces: the opened image, read
back, equals the bytes saved, for a classic bank, a compact bank and an
rbloom filter; doc slices equal the file's byte columns cut on the host.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bank_mod():
    from xspect2_amd import _lib
    from xspect2_amd import bank as bank_mod
    assert _lib.device_count() >= 1, "no HIP device visible"
    return bank_mod


def _roundtrip(bank_mod, b, tmp_path, kind, name):
    rng = np.random.default_rng(sum(name.encode()))
    payload = rng.integers(0, 256, b.payload_bytes(), dtype=np.uint8)
    b.upload(payload)
    path = tmp_path / name
    b.save(path)
    b.close()
    got = bank_mod.Bank.open(path, kind, device=0)
    try:
        assert np.array_equal(got.download(), payload)
    finally:
        got.close()
    return path, payload


def test_classic_file_over_many_pieces(bank_mod, tmp_path):
    """100 docs (13-B rows padded to 16 on the device), 9,000,011 rows:
    117 MB of payload, 3.5 pieces; then doc slices of it."""
    from xspect2_amd._lib import XS_BANK_COBS_CLASSIC
    D, S = 100, 9_000_011
    b = bank_mod.Bank.create_cobs(21, 7, [S], D, [f"d{i}" for i in range(D)])
    path, payload = _roundtrip(bank_mod, b, tmp_path, XS_BANK_COBS_CLASSIC, "big.cobs_classic")
    rows = payload.reshape(S, 13)
    for lo, hi in ((0, 8), (8, 64), (96, 100), (0, 100)):
        sl = bank_mod.Bank.open(path, XS_BANK_COBS_CLASSIC, device=0, docs=(lo, hi))
        try:
            # the open staged one ~32 MiB piece of whole rows at a time, never the whole 117 MB
            # of rows (config 5's split is for banks one GPU cannot hold), and kept none
            held, peak = sl.workspace_bytes()
            assert held == 0 and 0 < peak <= 33 << 20 < S * 13, (lo, hi, held, peak)
            want = np.ascontiguousarray(rows[:, lo // 8: lo // 8 + (hi - lo + 7) // 8])
            assert np.array_equal(sl.download(), want.reshape(-1)), (lo, hi)
        finally:
            sl.close()


def test_compact_file_over_many_pieces(bank_mod, tmp_path):
    """A compact bank of 3 groups (64-B rows) of different signature sizes:
    ~105 MB of payload."""
    from xspect2_amd._lib import XS_BANK_COBS_COMPACT
    D = 1430
    b = bank_mod.Bank.create_cobs(31, 1, [700_001, 500_003, 440_009], D, [f"a{i}" for i in range(D)],
                                  page_size=64, compact=True)
    _roundtrip(bank_mod, b, tmp_path, XS_BANK_COBS_COMPACT, "big.cobs_compact")


def test_rbloom_file_over_many_pieces(bank_mod, tmp_path):
    """An rbloom filter of 100 MB + 7 bytes."""
    from xspect2_amd._lib import XS_BANK_RBLOOM
    b = bank_mod.Bank.create_bloom(21, 100_000_007, 7)
    _roundtrip(bank_mod, b, tmp_path, XS_BANK_RBLOOM, "big.bloom")


def test_failed_save_leaves_the_existing_file(bank_mod, tmp_path):
    """xs_bank_save writes beside the destination and renames the file over it
    once whole: a save that fails (here: the temporary name is
    taken by a directory) returns an error and leaves the model already at
    the path byte for byte, with no partial file; a save that succeeds
    replaces it and leaves nothing else behind."""
    import os

    from xspect2_amd import _lib
    from xspect2_amd._lib import XS_BANK_COBS_CLASSIC
    D, S = 100, 300_007
    b = bank_mod.Bank.create_cobs(21, 7, [S], D, [f"d{i}" for i in range(D)])
    rng = np.random.default_rng(5)
    old = rng.integers(0, 256, b.payload_bytes(), dtype=np.uint8)
    b.upload(old)
    path = tmp_path / "m.cobs_classic"
    b.save(path)
    before = path.read_bytes()
    new = rng.integers(0, 256, b.payload_bytes(), dtype=np.uint8)
    b.upload(new)
    blocker = tmp_path / f"m.cobs_classic.xs-part-{os.getpid()}"
    blocker.mkdir()
    rc = _lib.load().xs_bank_save(b.handle, str(path).encode())
    assert rc == _lib.XS_ERR_IO, rc
    assert path.read_bytes() == before
    blocker.rmdir()
    b.save(path)
    assert sorted(p.name for p in tmp_path.iterdir()) == ["m.cobs_classic"]
    got = bank_mod.Bank.open(path, XS_BANK_COBS_CLASSIC, device=0)
    try:
        assert np.array_equal(got.download(), new)
    finally:
        got.close()
        b.close()
