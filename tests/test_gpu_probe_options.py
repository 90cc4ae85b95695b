"""Per-handle probe path selection (xs_bank_set_probe_options, GPU).

Round 5 chose the partitioned paths, the workspace cap and the small-call
path from environment variables read on every call; tests flipped them with
setenv while the library's worker threads ran, and an inherited environment
could put a production query on a test path.  They are
now options of the bank handle: the defaults are the production paths, the
old variables change nothing, and every path gives the same answer.
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


DEFAULTS = {"cobs_part": 1, "bloom_part": 1, "workspace_mib": 24 << 10, "small_calls": 1}


def test_defaults_roundtrip_and_bad_values(bank_mod):
    from xspect2_amd._lib import XsError
    b = bank_mod.Bank.create_cobs(21, 7, [1001], 10)
    try:
        assert b.probe_options() == DEFAULTS
        assert b.set_probe_options(cobs_part=3, workspace_mib=2) == DEFAULTS
        assert b.probe_options() == {**DEFAULTS, "cobs_part": 3, "workspace_mib": 2}
        for bad in ({"cobs_part": 5}, {"cobs_part": -1}, {"bloom_part": 4}, {"workspace_mib": 0},
                    {"small_calls": 2}):
            with pytest.raises(XsError):
                b.set_probe_options(**bad)
        with pytest.raises(TypeError):
            b.set_probe_options(lookup=1)
        assert b.probe_options() == {**DEFAULTS, "cobs_part": 3, "workspace_mib": 2}  # refused: unchanged
        b2 = bank_mod.Bank.create_bloom(21, 4096, 7)
        assert b2.probe_options() == DEFAULTS  # per handle
        b2.close()
    finally:
        b.close()


def test_environment_does_not_select_paths(bank_mod, monkeypatch):
    """A 48 MB classic bank and a call of 70 k reads (> 2^23 k-mers): the
    default options take the partitioned probe even with round 5's variables
    set to their 'off' values in the environment; the handle's option takes
    the direct probe; the two answers are equal, and the small-call option
    likewise changes the path of a 10-read call, not its answer."""
    from xspect2_amd import _lib
    for var, val in (("XSPECT2_AMD_COBS_PART", "0"), ("XSPECT2_AMD_BLOOM_PART", "0"),
                     ("XSPECT2_AMD_CP_WS_MB", "1"), ("XSPECT2_AMD_SMALL", "0")):
        monkeypatch.setenv(var, val)
    D, S = 100, 3_000_017
    rng = np.random.default_rng(11)
    rows = np.frombuffer(rng.bytes(S * 13), np.uint8) | np.frombuffer(rng.bytes(S * 13), np.uint8)
    rows = rows.reshape(S, 13).copy()
    rows[:, 12] &= 0x0F
    b = bank_mod.Bank.create_cobs(21, 7, [S], D)
    try:
        b.upload(rows.reshape(-1))
        acgt = np.frombuffer(b"ACGT", np.uint8)
        reads = [acgt[rng.integers(0, 4, 150)].tobytes() for _ in range(70_000)]
        part_h, part_n = b.query(reads)
        assert b.probe_path() == _lib.XS_PATH_PARTITIONED
        b.set_probe_options(cobs_part=0)
        direct_h, direct_n = b.query(reads)
        assert b.probe_path() == _lib.XS_PATH_GATHER
        assert np.array_equal(part_h, direct_h) and np.array_equal(part_n, direct_n)
        assert int(part_h.sum()) > 0
        few = reads[:10]
        want = b.query(few)[0]
        b.set_probe_options(small_calls=0)
        assert np.array_equal(b.query(few)[0], want) and np.array_equal(want, direct_h[:10])
    finally:
        b.close()
