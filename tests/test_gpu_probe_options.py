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
    """A 48 MB classic bank and one device call of 70 k reads (> 2^23
    k-mers): the default options take the partitioned probe even with round
    5's variables set to their 'off' values in the environment; the handle's
    option takes the direct probe; the two answers are equal, and the
    small-call option likewise changes the path of a 10-read call, not its
    answer."""
    torch = pytest.importorskip("torch")
    from xspect2_amd import _lib
    for var, val in (("XSPECT2_AMD_COBS_PART", "0"), ("XSPECT2_AMD_BLOOM_PART", "0"),
                     ("XSPECT2_AMD_CP_WS_MB", "1"), ("XSPECT2_AMD_SMALL", "0")):
        monkeypatch.setenv(var, val)
    D, S, n, L = 100, 3_000_017, 70_000, 150
    rng = np.random.default_rng(11)
    rows = np.frombuffer(rng.bytes(S * 13), np.uint8) | np.frombuffer(rng.bytes(S * 13), np.uint8)
    rows = rows.reshape(S, 13).copy()
    rows[:, 12] &= 0x0F
    b = bank_mod.Bank.create_cobs(21, 7, [S], D)
    try:
        b.upload(rows.reshape(-1))
        reads = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, n * L)]
        dev = torch.device("cuda", 0)
        d_seq = torch.from_numpy(reads.copy()).to(dev)
        d_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
        s = torch.cuda.current_stream(dev).cuda_stream

        def probe():
            hits = torch.empty((n, D), dtype=torch.int32, device=dev)
            tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
            b.query_device(d_seq, n * L, d_off, n, 1, hits, None, tot, stream=s)
            torch.cuda.synchronize(dev)
            return hits.cpu().numpy(), tot.cpu().numpy(), b.probe_path()

        part_h, part_t, path = probe()
        assert path == _lib.XS_PATH_PARTITIONED
        b.set_probe_options(cobs_part=0)
        direct_h, direct_t, path = probe()
        assert path == _lib.XS_PATH_GATHER
        assert np.array_equal(part_h, direct_h) and np.array_equal(part_t, direct_t) and int(part_t[:D].sum()) > 0
        few = [reads[i * L:(i + 1) * L].tobytes() for i in range(10)]
        want = b.query(few)[0]
        b.set_probe_options(small_calls=0)
        assert np.array_equal(b.query(few)[0], want) and np.array_equal(want, direct_h[:10].view(np.uint32))
    finally:
        b.close()


def test_options_change_while_other_threads_query(bank_mod, oracle_mod):
    """One thread flips the handle's probe options (direct / partitioned COBS,
    small calls on / off, 1-4 MiB workspaces) while three others query the
    same handle: every answer equals the oracle's (options apply between
    queries, under the handle's mutex; round 5's setenv could race the
    library's getenv on worker threads)."""
    import threading

    from test_gpu_parity import _pair, _reads
    ob, gb, seqs, _ = _pair(bank_mod, oracle_mod, 100, 21, 7, [30_011], seed=21)
    rng = np.random.default_rng(21)
    genome = b"".join(seqs)
    sets = []
    for n in (5, 300, 3000, 9000):
        reads = [genome[o:o + 150] for o in rng.integers(0, len(genome) - 150, n)] + _reads(rng, 20, 21)
        sets.append((reads, ob.query(reads)))
    stop, errors = threading.Event(), []

    def flip():
        i = 0
        while not stop.is_set():
            gb.set_probe_options(cobs_part=(0, 2, 3)[i % 3], small_calls=i % 2, workspace_mib=1 + i % 4)
            i += 1

    def work(t):
        try:
            for rep in range(6):
                reads, (want_h, want_n) = sets[(t + rep) % len(sets)]
                got_h, got_n = gb.query(reads)
                if not (np.array_equal(got_h, want_h) and np.array_equal(got_n, want_n)):
                    errors.append(f"thread {t} rep {rep}: mismatch")
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    flipper = threading.Thread(target=flip)
    workers = [threading.Thread(target=work, args=(t,)) for t in range(3)]
    flipper.start()
    for w in workers:
        w.start()
    for w in workers:
        w.join()
    stop.set()
    flipper.join()
    gb.close()
    assert not errors, errors
