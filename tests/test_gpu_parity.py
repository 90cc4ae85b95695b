"""Parity of the HIP probe path with the CPU oracle, through the C ABI (GPU).

Bit-exact for every integer output: hit matrices, k-mer counts, totals and
the bank images built on the device.  Inputs are seeded; edge cases follow
what the reference's path meets: reads of length <= k (no k-mers), exactly
k+1, non-ACGT bytes (N, IUPAC, lower case), long records split into several
work units, sparse sampling steps, empty reads, D spanning 1..1000 docs.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def xs():
    from xspect2_amd import bank as bank_mod
    from xspect2_amd import _lib
    assert _lib.device_count() >= 1, "no HIP device visible"
    return bank_mod


def _reads(rng, n, k, alphabet="ACGT", min_len=None, max_len=300):
    lo = min_len if min_len is not None else max(0, k - 2)
    alph = np.frombuffer(alphabet.encode(), dtype=np.uint8)
    return [alph[rng.integers(0, alph.size, int(L))].tobytes() for L in rng.integers(lo, max_len, n)]


def _docs(rng, D, k, per_doc=2, max_len=2000):
    seqs, ids = [], []
    for d in range(D):
        for _ in range(per_doc):
            L = int(rng.integers(k, max_len))
            seqs.append(np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)].tobytes())
            ids.append(d)
    return seqs, ids


def _pair(xs, oracle_mod, D, k, h, sig, page=None, seed=0, per_doc=2):
    """Oracle bank and device bank holding the same image."""
    rng = np.random.default_rng(seed)
    seqs, ids = _docs(rng, D, k, per_doc)
    compact = page is not None
    P = page if compact else (D + 7) // 8
    ob = oracle_mod.CobsBank.empty(sig, P, D, h, k)
    ob.build(seqs, ids)
    gb = xs.Bank.create_cobs(k, h, sig, D, [f"doc{i}" for i in range(D)],
                             page_size=P if compact else None, compact=compact)
    gb.upload(ob.rows)
    return ob, gb, seqs, ids


CLASSIC_CASES = [
    # D, k, h, sig
    (1, 21, 7, [997]),
    (3, 21, 7, [5000]),
    (8, 5, 2, [301]),
    (100, 21, 7, [40_000]),
    (129, 31, 1, [20_011]),
    (300, 16, 3, [7_919]),
    (1000, 21, 7, [3_001]),
    (13, 32, 4, [2_048]),
    (40, 17, 9, [1_231]),
    (200, 21, 7, [12_007]),   # wide kernel, 2 chunk lanes
    (500, 31, 1, [9_001]),    # wide kernel, 4 chunk lanes
    (700, 25, 5, [4_001]),    # wide kernel, 8 chunk lanes, general (k, h)
    (2048, 31, 1, [9_001]),   # wide kernel, 16 chunk lanes (rows of two lines)
    (2000, 21, 7, [6_007]),   # wide kernel, 16 chunk lanes, species (k, h)
    (1100, 16, 3, [3_011]),   # wide kernel, 9 data chunks of 16 lanes, general (k, h)
    (2100, 21, 7, [4_001]),   # 17 chunks: general kernel
]


@pytest.mark.parametrize("D,k,h,sig", CLASSIC_CASES)
def test_classic_probe_matches_oracle(xs, oracle_mod, D, k, h, sig):
    _classic_case(xs, oracle_mod, D, k, h, sig, opts={"cobs_part": 0})


@pytest.mark.parametrize("D,k,h,sig", [c for c in CLASSIC_CASES if c[0] <= 128] + [(128, 21, 7, [70_001]),
                                                                                  (64, 31, 8, [300_007])])
@pytest.mark.parametrize("mode,ws_mb", [("3", None), ("3", "1"), ("3", "2"), ("4", None), ("4", "2")])
def test_classic_partitioned_probe_matches_oracle(xs, oracle_mod, D, k, h, sig, mode, ws_mb):
    """The partitioned COBS probe (k-mer rows binned by bank partition, per-XCD
    L2-resident lookup, per-block AND + count) with partitions down to 1024
    rows (mode 3) or of exactly 1024 rows (mode 4: banks over 512 Ki rows get
    more than 512 partitions, whose runs are not padded), and workspaces of
    1-2 MiB (the bucket blocks then run in ranges of a few blocks that reuse
    it), on the classic cases of <= 128 docs: same hits, counts and totals."""
    _classic_case(xs, oracle_mod, D, k, h, sig, want_path=1 if h <= 8 else 0, opts=_opts(mode, ws_mb))


def _random_partitioned_configs(n=48, seed=20261017):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        D = int(rng.integers(1, 129))
        k = int(rng.integers(5, 33))
        h = int(rng.integers(1, 9))
        sig = int(rng.integers(1_000, 200_001))
        mode = str(int(rng.choice([3, 4])))
        ws_mb = [None, "1", "2"][int(rng.integers(0, 3))]
        out.append((D, k, h, sig, mode, ws_mb))
    return out


@pytest.mark.parametrize("D,k,h,sig,mode,ws_mb", _random_partitioned_configs())
def test_partitioned_probe_random_configs(xs, oracle_mod, D, k, h, sig, mode, ws_mb):
    """Seeded random configurations of the partitioned COBS probe (docs 1-128,
    k 5-32, h 1-8, 1 k-200 k rows in partitions down to 1024 rows or of 1024
    rows, small workspaces that force block ranges, padded and unpadded runs):
    same hits, k-mer counts and totals as the oracle at steps 1, 2 and 7."""
    _classic_case(xs, oracle_mod, D, k, h, [sig], want_path=1, opts=_opts(mode, ws_mb))


@pytest.mark.parametrize("mode,D", [("4", 100), ("4", 117), ("4", 128), ("3", 64), ("3", 128)])
def test_partitioned_padding_threshold(xs, oracle_mod, mode, D):
    """A 1 M-row bank cut into 1024-row partitions (mode 4: 977 of them, more
    than kCobsPadParts = 512, so the runs are not padded) and into 64
    partitions (mode 3: padded with all-ones pad rows), with the k-mer id in
    the row's top bits (D <= 117) and in the entries (D = 128): same hits,
    counts and totals as the oracle."""
    _classic_case(xs, oracle_mod, D, 21, 7, [1_000_003], want_path=1, opts=_opts(mode))


def test_partitioned_largest_partitions(xs, oracle_mod):
    """A bank of 2^27 + 15 rows (2 GiB on the device): 1025 partitions of 2^17
    rows would exceed kPartMax = 1024, so the plan doubles them to 2^18 rows
    (513 partitions: more than kCobsPadParts, unpadded runs); same hits as
    the oracle."""
    _classic_case(xs, oracle_mod, 100, 21, 7, [(1 << 27) + 15], want_path=1, opts={"cobs_part": 2})


def _opts(mode, ws_mb=None):
    """Probe options of a parametrised case: cobs_part mode, optional workspace cap in MiB."""
    o = {"cobs_part": int(mode)}
    if ws_mb:
        o["workspace_mib"] = int(ws_mb)
    return o


def _classic_case(xs, oracle_mod, D, k, h, sig, want_path=None, opts=None):
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, seed=D * 31 + k)
    if opts:
        gb.set_probe_options(**opts)
    rng = np.random.default_rng(D + k + h)
    reads = _reads(rng, 300, k)
    reads += [s[: int(rng.integers(k, len(s) + 1))] for s in seqs[:40]]      # true positives
    reads += _reads(rng, 40, k, alphabet="ACGTNacgtnRYKM")                   # non-ACGT
    reads += [b"", b"A" * (k - 1) if k > 1 else b"", b"C" * k, b"G" * (k + 1)]
    reads += [seqs[0] * 3]                                                   # multi-unit read
    for step in (1, 2, 7):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n), f"num_kmers differ (step {step})"
        assert np.array_equal(got_h, want_h), _explain(got_h, want_h, reads)
        if want_path is not None:
            assert gb.probe_path() == want_path
        tot, nk = gb.query_totals(reads, step=step)
        assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64))
        assert nk == int(want_n.sum())
    gb.close()


@pytest.mark.parametrize("case", ["all_short", "one_read", "one_long_read", "empty_only", "tiny_reads",
                                  "empty_between"])
def test_partitioned_degenerate_batches(xs, oracle_mod, case):
    """Forced partitioned COBS probe on batches with no k-mers at all, a single
    read, a single read spanning many bucket blocks, only empty reads, reads
    of 1-3 k-mers (a bucket block spans more reads than it stages in LDS) and
    reads with runs of empty and short reads between them (reads sharing a
    first k-mer in the block's k-mer -> read map): hits, counts and totals
    equal the oracle's (zeros where no k-mer)."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=12)
    gb.set_probe_options(cobs_part=3)
    rng = np.random.default_rng(5)
    genome = b"".join(seqs)

    def cut(n, lo, hi):
        out = []
        for _ in range(n):
            L = int(rng.integers(lo, hi + 1))
            o = int(rng.integers(0, len(genome) - L))
            out.append(genome[o:o + L])
        return out

    mixed = []
    for r in cut(400, 60, 300):
        mixed += [b""] * int(rng.integers(0, 4)) + [b"ACGT"[: int(rng.integers(0, 4))]] + [r]
    reads = {"all_short": _reads(rng, 500, 21, min_len=0, max_len=21),
             "one_read": [seqs[0][:150]],
             "one_long_read": [b"".join(seqs[:4])[:20_000]],
             "empty_only": [b""] * 7,
             "tiny_reads": cut(6000, 21, 23),
             "empty_between": mixed}[case]
    for step in (1, 2):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n) and np.array_equal(got_h, want_h)
        tot, nk = gb.query_totals(reads, step=step)
        assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
    gb.close()


def test_partitioned_default_on_bank_over_mall(xs, oracle_mod):
    """Default mode on a classic bank larger than the Infinity Cache (17 M
    rows x 16 B = 272 MB on the device): the query takes the partitioned path
    by itself; host and device APIs, totals, best doc, steps 1 and 3, reads of
    every length class (empty, < k, one unit, several units), bit-exact;
    then once more in ranges reusing a 64 MiB workspace."""
    torch = pytest.importorskip("torch")
    from xspect2_amd import _lib
    from xspect2_amd.packing import pack_sequences
    D, k, h, sig = 100, 21, 7, 17_000_011
    rng = np.random.default_rng(2024)
    nb = sig * 13
    rows = (np.frombuffer(rng.bytes(nb), np.uint8) | np.frombuffer(rng.bytes(nb), np.uint8)
            | np.frombuffer(rng.bytes(nb), np.uint8))  # ~7/8 of the bits set: AND of 7 rows ~0.39
    rows = rows.reshape(sig, 13).copy()
    rows[:, 12] &= 0x0F  # docs 100..103 do not exist
    ob = oracle_mod.CobsBank(rows.reshape(-1), [sig], 13, D, h, k)
    gb = xs.Bank.create_cobs(k, h, [sig], D, [f"d{i}" for i in range(D)])
    gb.upload(ob.rows)
    reads = _reads(rng, 60_000, k, min_len=140, max_len=160)  # > 2^23 k-mers: the default takes the path
    reads += _reads(rng, 300, k, alphabet="ACGTacgtNRY", min_len=0, max_len=400)
    reads += [b"", b"A" * (k - 1), _reads(rng, 1, k, min_len=5000, max_len=5001)[0]]
    want = {}
    for step in (1, 3):
        want_h, want_n = ob.query(reads, step=step)
        want[step] = (want_h, want_n)
        # host batches go in 8/32 MiB chunks, some under the default's k-mer
        # threshold (step 3 always): force the path so every chunk takes it
        gb.set_probe_options(cobs_part=2)
        got_h, got_n = gb.query(reads, step=step)
        assert gb.probe_path() == _lib.XS_PATH_PARTITIONED
        gb.set_probe_options(cobs_part=1)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h, want_h), int((got_h != want_h).sum())
        tot, nk = gb.query_totals(reads, step=step)
        assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
        best, bh, bnk, btot = gb.query_best(reads, step=step, want_totals=True)
        assert np.array_equal(bh, want_h.max(axis=1)) and np.array_equal(bnk, want_n)
    assert 0 < int(want_h.sum())
    gb.set_probe_options(workspace_mib=64)
    got_h, got_n = gb.query(reads, step=3)
    assert np.array_equal(got_h, want_h) and np.array_equal(got_n, want_n)
    gb.set_probe_options(workspace_mib=24 << 10)
    # device API on a torch stream
    pr = pack_sequences(reads)
    dev = torch.device("cuda", 0)
    d_seq = torch.from_numpy(pr.buf.copy()).to(dev)
    d_off = torch.from_numpy(pr.offsets.astype(np.int64)).to(dev)
    d_hits = torch.empty((pr.n, D), dtype=torch.int32, device=dev)
    d_nk = torch.empty(pr.n, dtype=torch.int64, device=dev)
    d_tot = torch.empty(D + 1, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    gb.query_device(d_seq, int(pr.offsets[-1]), d_off, pr.n, 1, d_hits, d_nk, d_tot, stream=st.cuda_stream)
    st.synchronize()
    assert gb.probe_path() == _lib.XS_PATH_PARTITIONED  # one call of 60 k reads: over the default threshold
    want_h, want_n = want[1]
    assert np.array_equal(d_hits.cpu().numpy().view(np.uint32), want_h)
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert np.array_equal(tot[:D], want_h.sum(axis=0, dtype=np.uint64)) and int(tot[D]) == int(want_n.sum())
    gb.close()


@pytest.mark.parametrize("D,k,h,page,G", [(600, 31, 1, 64, 2), (20, 21, 7, 1, 3), (1500, 21, 2, 64, 3),
                                          (70, 25, 3, 3, 3), (2600, 31, 1, 64, 6), (1430, 31, 1, 64, 3),
                                          (600, 31, 1, 32, 3), (100, 21, 3, 2, 7), (2000, 31, 1, 64, 4),
                                          (700, 31, 1, 40, 3), (500, 21, 7, 48, 2)])
def test_compact_probe_matches_oracle(xs, oracle_mod, D, k, h, page, G):
    assert (G - 1) * 8 * page < D <= G * 8 * page
    rng = np.random.default_rng(D)
    sig = [int(x) for x in rng.integers(500, 6000, G)]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, page=page, seed=D, per_doc=1)
    reads = _reads(rng, 200, k) + [s[:300] for s in seqs[:50]] + _reads(rng, 20, k, "ACGTN")
    for step in (1, 3):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h, want_h)
    gb.close()


@pytest.mark.parametrize("D,k,G", [(1430, 31, 3), (1025, 31, 3), (1536, 31, 3), (2048, 31, 4), (1537, 21, 4),
                                   (1300, 15, 3), (1800, 32, 4), (400, 31, 1), (512, 31, 1), (70, 31, 1),
                                   (300, 21, 1), (900, 31, 2), (513, 31, 2), (1024, 17, 2)])
def test_vslice_probe_matches_oracle(xs, oracle_mod, D, k, G):
    """Compact banks of 1-4 groups of 64-byte pages with one hash (MLST loci)
    take the bit-sliced probe (xs_probe_vslice.hip; 4 or 2 k-mer slots per
    wave at 1 or 2 groups): hits, k-mer counts and totals equal the oracle's
    for random and document reads, reads of exactly 256 k-mers from one
    document (a count of 256: the weight-256 plane at 3-4 groups, the slots'
    sum at 1-2), reads of two full units, non-ACGT, empty and short reads, at
    steps 1 and 3."""
    rng = np.random.default_rng(D + 7 * k)
    sig = [int(x) for x in rng.integers(3000, 40000, G)]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, 1, sig, page=64, seed=D + k, per_doc=1)
    long_docs = [s for s in seqs if len(s) >= 600]
    assert len(long_docs) >= 20
    reads = _reads(rng, 200, k) + [s[: int(rng.integers(k, len(s) + 1))] for s in seqs[:60]]
    reads += [s[: 255 + k] for s in long_docs[:10]]   # 256 k-mers at step 1: one whole unit
    reads += [s[: 511 + k] for s in long_docs[10:20]]  # two full units
    reads += _reads(rng, 20, k, alphabet="ACGTNacgtnRY") + [b"", b"A" * (k - 1), seqs[0] * 3]
    for step in (1, 3):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h, want_h), _explain(got_h, want_h, reads)
        tot, nk = gb.query_totals(reads, step=step)
        assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
        if step == 1:
            assert int(want_h.max()) >= 256
    gb.close()


def _random_direct_configs(n=32, seed=20261018):
    """Seeded random banks for the direct COBS probe families (fast, wide,
    slots, general): classic with 1..2200 docs, or compact with page sizes
    1..64 and 1..8 groups; k 5..32, h 1..9; a few thousand rows per group."""
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k = int(rng.integers(5, 33))
        h = int(rng.integers(1, 10))
        if rng.random() < 0.5:
            D = int(rng.choice([int(rng.integers(1, 129)), int(rng.integers(129, 2201))]))
            out.append((D, k, h, None, 1))
        else:
            page = int(rng.choice([1, 2, 3, 8, 16, 32, 40, 48, 64]))
            G = int(rng.integers(1, 9))
            D = int(rng.integers((G - 1) * 8 * page + 1, G * 8 * page + 1))
            out.append((D, k, h, page, G))
    return out


@pytest.mark.parametrize("D,k,h,page,G", _random_direct_configs())
def test_direct_probe_random_configs(xs, oracle_mod, D, k, h, page, G):
    """Seeded random classic and compact banks through the direct probes
    (the partitioned path kept off): same hits, k-mer counts and totals as
    the oracle at steps 1 and 4, for random, document-derived, non-ACGT,
    short and multi-unit reads."""
    rng = np.random.default_rng(D * 131 + k * 7 + h)
    sig = [int(x) for x in rng.integers(700, 5000, G)]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, page=page, seed=D + k, per_doc=1)
    gb.set_probe_options(cobs_part=0)
    reads = _reads(rng, 150, k) + [s[: int(rng.integers(k, len(s) + 1))] for s in seqs[:40]]
    reads += _reads(rng, 20, k, alphabet="ACGTNacgtnRY") + [b"", b"A" * max(k - 1, 0), seqs[0] * 3]
    for step in (1, 4):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h, want_h), _explain(got_h, want_h, reads)
        tot, nk = gb.query_totals(reads, step=step)
        assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
    gb.close()


def _random_build_configs(n=16, seed=20261019):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        k, h = int(rng.integers(5, 33)), int(rng.integers(1, 10))
        page = None if rng.random() < 0.5 else int(rng.choice([1, 2, 8, 64]))
        D = int(rng.integers(1, 300))
        out.append((D, k, h, page))
    return out


@pytest.mark.parametrize("D,k,h,page", [(5, 21, 7, None), (100, 21, 7, None), (37, 31, 1, 2), (12, 32, 3, None)]
                         + _random_build_configs())
def test_device_build_matches_oracle_build(xs, oracle_mod, D, k, h, page):
    rng = np.random.default_rng(7 * D + k)
    seqs, ids = _docs(rng, D, k, per_doc=3)
    seqs += _reads(rng, 5, k, "ACGTNacgtRY")
    ids += [int(rng.integers(0, D)) for _ in range(5)]
    compact = page is not None
    P = page if compact else (D + 7) // 8
    G = 1 if not compact else (D + 8 * P - 1) // (8 * P)
    sig = [int(x) for x in rng.integers(300, 5000, G)]
    ob = oracle_mod.CobsBank.empty(sig, P, D, h, k)
    ob.build(seqs, ids)
    gb = xs.Bank.create_cobs(k, h, sig, D, page_size=P if compact else None, compact=compact)
    gb.build(seqs, ids)
    assert np.array_equal(gb.download(), ob.rows)
    gb.close()


def test_bank_file_roundtrip(xs, oracle_mod, tmp_path):
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 10, 21, 7, [4099], seed=3)
    path = tmp_path / "m" / "index.cobs_classic"
    gb.save(path)
    gb2 = xs.Bank.open(path, xs.XS_BANK_COBS_CLASSIC)
    assert gb2.doc_names == [f"doc{i}" for i in range(10)]
    assert np.array_equal(gb2.download(), ob.rows)
    reads = [s[:150] for s in seqs]
    assert np.array_equal(gb2.query(reads)[0], ob.query(reads)[0])
    gb.close()
    gb2.close()


@pytest.mark.parametrize("mode", ["0", "3"])
@pytest.mark.parametrize("k", [21, 31, 5, 16, 32])
def test_bloom_probe_and_build_match_oracle(xs, oracle_mod, k, mode):
    """mode 0: direct probe; mode 3: partitioned probe with small partitions."""
    rng = np.random.default_rng(k)
    genome = _reads(rng, 6, k, alphabet="ACGTacgtN", min_len=k, max_len=3000)
    n_items = sum(len(s) for s in genome) - k + 1
    nbytes, K = oracle_mod.BloomFilter.params(n_items, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(genome)
    gb = xs.Bank.create_bloom(k, nbytes, K)
    gb.set_probe_options(bloom_part=int(mode))
    gb.build(genome)
    assert np.array_equal(gb.download(), bf.bits), "device-built filter differs"
    reads = _reads(rng, 300, k, alphabet="ACGTacgtNRY") + [g[:500] for g in genome] + [genome[0]]
    for step in (1, 4):
        want_h, want_n = bf.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h[:, 0], want_h)
        tot, nk = gb.query_totals(reads, step=step)
        assert int(tot[0]) == int(want_h.sum()) and nk == int(want_n.sum())
    gb.close()


def _random_bloom_configs(n=24, seed=1017):
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(5, 33)), int(rng.integers(1_000, 2_000_001)), int(rng.integers(1, 9)),
             int(rng.integers(0, 1_000_000))) for _ in range(n)]


@pytest.mark.parametrize("k,nbytes,K,seed", _random_bloom_configs())
def test_bloom_partitioned_random_configs(xs, oracle_mod, k, nbytes, K, seed):
    """Seeded random rbloom filters (k 5-32, 1 kB-2 MB, K 1-8 bit indices)
    through the partitioned probe with small partitions; mixed-case / IUPAC
    reads: same hits, counts and totals as the oracle at steps 1 and 3."""
    rng = np.random.default_rng(seed)
    genome = _reads(rng, 8, k, alphabet="ACGTacgtN", min_len=k, max_len=5000)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(genome)
    gb = xs.Bank.create_bloom(k, nbytes, K)
    gb.set_probe_options(bloom_part=3)
    gb.build(genome)
    assert np.array_equal(gb.download(), bf.bits), "device-built filter differs"
    reads = _reads(rng, 400, k, alphabet="ACGTacgtNRY") + [g[:300] for g in genome] + [genome[0] * 2]
    for step in (1, 3):
        want_h, want_n = bf.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h[:, 0], want_h)
        assert gb.probe_path() == 1
        tot, nk = gb.query_totals(reads, step=step)
        assert int(tot[0]) == int(want_h.sum()) and nk == int(want_n.sum())
    gb.close()


@pytest.mark.parametrize("mode", ["0", "3"])
@pytest.mark.parametrize("k", [21, 31])
def test_bloom_single_odd_byte_at_every_window_position(xs, oracle_mod, k, mode):
    """Uppercase ACGT reads with one N, lower-case or IUPAC byte: the read is
    2k-1 long with the odd byte in the middle, so its k windows hold that byte
    at every window position 0..k-1.  Windows with an N take the permute
    complement, the others the per-byte Biopython table; half the reads are in
    the filter, so hits are non-trivial.  Both probe paths."""
    rng = np.random.default_rng(k + 5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    odd = b"NnacgtRYKMSWBDHVXU-*."
    reads = []
    for rep in range(4):
        for c in odd:
            r = bytearray(acgt[rng.integers(0, 4, 2 * k - 1)].tobytes())
            r[k - 1] = c
            reads.append(bytes(r))
    members = reads[::2]
    bf = oracle_mod.BloomFilter(np.zeros(50_021, dtype=np.uint8), 7, k)
    bf.build(members)
    gb = xs.Bank.create_bloom(k, 50_021, 7)
    gb.set_probe_options(bloom_part=int(mode))
    gb.build(members)
    assert np.array_equal(gb.download(), bf.bits), "device-built filter differs"
    want_h, want_n = bf.query(reads)
    got_h, got_n = gb.query(reads)
    assert np.array_equal(got_n, want_n)
    assert np.array_equal(got_h[:, 0], want_h)
    assert int(want_h[::2].sum()) == k * len(members)  # every window of a member read is a member


@pytest.mark.parametrize("mode,k,K,nbytes", [("3", 21, 7, 200_003), ("3", 31, 5, 77_777), ("3", 16, 8, 1 << 20),
                                             ("1", 21, 7, 40 << 20), ("1", 21, 7, (1 << 31) + 4099),
                                             ("3", 21, 10, 100_003)])  # K > 8: gather path
def test_bloom_partitioned_probe_matches_oracle(xs, oracle_mod, mode, k, K, nbytes):
    """The partitioned rbloom probe (k-mer bit indices binned by filter
    partition, per-partition lookup, per-read count) against the oracle:
    hundreds of bucket blocks, ragged and multi-unit reads, empty and short
    reads, non-ACGT bytes, steps 1 and 3.  mode 1 with 40 MiB takes the
    default path (20 partitions of 2 MiB); the 2 GiB + 4 KiB filter needs
    4 MiB partitions (more than 1024 of 2 MiB) and a partial last one."""
    rng = np.random.default_rng(nbytes % 1000 + k)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genome = [acgt[rng.integers(0, 4, 60_000)].tobytes() for _ in range(3)]
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(genome)
    gb = xs.Bank.create_bloom(k, nbytes, K)
    gb.set_probe_options(bloom_part=int(mode))
    gb.upload(bf.bits)
    reads = []
    for _ in range(2500):
        g = genome[int(rng.integers(0, 3))]
        st = int(rng.integers(0, len(g) - 200))
        reads.append(g[st:st + int(rng.integers(100, 200))])
    reads += _reads(rng, 800, k, alphabet="ACGT", max_len=400)
    reads += _reads(rng, 100, k, alphabet="ACGTacgtNRY")
    reads += [b"", b"A" * (k - 1), genome[1][:5000], b"", genome[2][:k], genome[0]]
    order = rng.permutation(len(reads))
    reads = [reads[i] for i in order]
    for step in (1, 3):
        want_h, want_n = bf.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n)
        assert np.array_equal(got_h[:, 0], want_h), int((got_h[:, 0] != want_h).sum())
        tot, nk = gb.query_totals(reads, step=step)
        assert int(tot[0]) == int(want_h.sum()) and nk == int(want_n.sum())
        best, bh, bnk, btot = gb.query_best(reads, step=step, want_totals=True)
        assert np.array_equal(bh, want_h) and np.array_equal(bnk, want_n)
        assert int(btot[0]) == int(want_h.sum()) and int(btot[1]) == int(want_n.sum())
    assert 0 < int(want_h.sum()) < int(want_n.sum())
    gb.close()


def test_bloom_partitioned_threads_and_torch_stream(xs, oracle_mod):
    """Partitioned probe from 4 host threads on one handle (serialised by its
    mutex) and on a second handle at once, then through the device API on a
    torch stream: every answer equals the oracle's."""
    import threading

    import torch
    rng = np.random.default_rng(44)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genome = [acgt[rng.integers(0, 4, 80_000)].tobytes()]
    nbytes = 20 << 20
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), 7, 21)
    bf.build(genome)
    banks = [xs.Bank.create_bloom(21, nbytes, 7) for _ in range(2)]
    for b in banks:
        b.set_probe_options(bloom_part=2)
        b.upload(bf.bits)
    sets = []
    for t in range(6):
        reads = [genome[0][s:s + 150] for s in rng.integers(0, 79_000, 3000)]
        reads += _reads(rng, 500, 21, min_len=100, max_len=200)
        sets.append((reads, bf.query(reads)))
    errors = []

    def work(b, items):
        try:
            for reads, (want_h, want_n) in items:
                got_h, got_n = b.query(reads)
                if not (np.array_equal(got_n, want_n) and np.array_equal(got_h[:, 0], want_h)):
                    errors.append("mismatch")
                if b.probe_path() != 1:
                    errors.append("path")
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=work, args=(banks[i % 2], sets[i::4])) for i in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
    # device API on a torch stream
    from xspect2_amd.packing import pack_sequences
    reads, (want_h, want_n) = sets[0]
    pr = pack_sequences(reads)
    dev = torch.device("cuda", 0)
    d_seq = torch.from_numpy(pr.buf.copy()).to(dev)
    d_off = torch.from_numpy(pr.offsets.astype(np.int64)).to(dev)
    d_hits = torch.empty((pr.n, 1), dtype=torch.int32, device=dev)
    d_nk = torch.empty(pr.n, dtype=torch.int64, device=dev)
    d_tot = torch.zeros(2, dtype=torch.int64, device=dev)
    st = torch.cuda.Stream(dev)
    banks[0].query_device(d_seq, d_seq.numel(), d_off, pr.n, 1, d_hits, d_nk, d_tot, stream=st.cuda_stream)
    st.synchronize()
    assert np.array_equal(d_hits.cpu().numpy()[:, 0].astype(np.uint32), want_h)
    assert np.array_equal(d_nk.cpu().numpy().astype(np.uint64), want_n)
    assert int(d_tot[0]) == int(want_h.sum()) and int(d_tot[1]) == int(want_n.sum())
    assert banks[0].probe_path() == 1
    for b in banks:
        b.close()


@pytest.mark.parametrize("step", [1, 2])
def test_bloom_partitioned_many_short_reads(xs, oracle_mod, step):
    """Bucket blocks spanning more reads than they stage in LDS (reads of
    k..k+3 bytes: 1-4 k-mers each, so a 1024-k-mer block holds hundreds of
    reads) take the global read search; mixed with empty and sub-k reads."""
    rng = np.random.default_rng(31 + step)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genome = [acgt[rng.integers(0, 4, 20_000)].tobytes()]
    bf = oracle_mod.BloomFilter(np.zeros(300_007, dtype=np.uint8), 7, 21)
    bf.build(genome)
    gb = xs.Bank.create_bloom(21, 300_007, 7)
    gb.set_probe_options(bloom_part=3)
    gb.upload(bf.bits)
    reads = []
    for _ in range(6000):
        L = int(rng.integers(15, 25))
        st = int(rng.integers(0, 19_000))
        reads.append(genome[0][st:st + L] if rng.random() < 0.6 else acgt[rng.integers(0, 4, L)].tobytes())
    reads[100:140] = [b""] * 40
    want_h, want_n = bf.query(reads, step=step)
    got_h, got_n = gb.query(reads, step=step)
    assert np.array_equal(got_n, want_n) and np.array_equal(got_h[:, 0], want_h)
    assert gb.probe_path() == 1
    gb.close()


@pytest.mark.parametrize("step", [1, 3])
def test_bloom_partitioned_empty_reads_between(xs, oracle_mod, step):
    """Reads of 60-300 bytes with runs of empty and sub-k reads between them:
    the bucket block stages its reads in LDS and several share a first k-mer
    in its k-mer -> read map (the later, non-empty one holds it)."""
    rng = np.random.default_rng(77 + step)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genome = acgt[rng.integers(0, 4, 50_000)].tobytes()
    bf = oracle_mod.BloomFilter(np.zeros(300_007, dtype=np.uint8), 7, 21)
    bf.build([genome])
    gb = xs.Bank.create_bloom(21, 300_007, 7)
    gb.set_probe_options(bloom_part=3)
    gb.upload(bf.bits)
    reads = []
    for _ in range(800):
        reads += [b""] * int(rng.integers(0, 4)) + [genome[:int(rng.integers(0, 21))]]
        L = int(rng.integers(60, 301))
        st = int(rng.integers(0, len(genome) - L))
        reads.append(genome[st:st + L] if rng.random() < 0.7 else acgt[rng.integers(0, 4, L)].tobytes())
    want_h, want_n = bf.query(reads, step=step)
    got_h, got_n = gb.query(reads, step=step)
    assert np.array_equal(got_n, want_n) and np.array_equal(got_h[:, 0], want_h)
    assert gb.probe_path() == 1
    gb.close()


def test_bloom_path_follows_member_fraction(xs, oracle_mod):
    """Default mode on a 40 MiB filter: the first query takes the partitioned
    path; after a member-poor query (random reads) the next takes the gather
    path, and after a member-rich one the partitioned path again.  Every
    answer equals the oracle's."""
    from xspect2_amd import _lib
    rng = np.random.default_rng(9)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genome = [acgt[rng.integers(0, 4, 50_000)].tobytes()]
    bf = oracle_mod.BloomFilter(np.zeros(40 << 20, dtype=np.uint8), 7, 21)
    bf.build(genome)
    gb = xs.Bank.create_bloom(21, 40 << 20, 7)
    gb.upload(bf.bits)
    members = [genome[0][s:s + 150] for s in rng.integers(0, 49_000, 2000)]
    foreign = _reads(rng, 2000, 21, alphabet="ACGT", min_len=150, max_len=151)
    paths = []
    for reads in (foreign, foreign, members, members):
        got_h, got_n = gb.query(reads)
        want_h, want_n = bf.query(reads)
        assert np.array_equal(got_n, want_n) and np.array_equal(got_h[:, 0], want_h)
        paths.append(gb.probe_path())
    P, G = _lib.XS_PATH_PARTITIONED, _lib.XS_PATH_GATHER
    assert paths == [P, G, G, P], paths
    gb.close()


def test_bloom_file_roundtrip(xs, oracle_mod, tmp_path):
    bits = np.random.default_rng(1).integers(0, 256, 4097, dtype=np.uint8)
    gb = xs.Bank.create_bloom(21, bits.size, 7)
    gb.upload(bits)
    gb.save(tmp_path / "filter.bloom")
    raw = (tmp_path / "filter.bloom").read_bytes()
    assert int.from_bytes(raw[:8], "little") == 7 and raw[8:] == bits.tobytes()
    gb2 = xs.Bank.open(tmp_path / "filter.bloom", xs.XS_BANK_RBLOOM, term_size=21)
    assert np.array_equal(gb2.download(), bits)
    bf = oracle_mod.BloomFilter(bits, 7, 21)
    reads = _reads(np.random.default_rng(2), 100, 21)
    assert np.array_equal(gb2.query(reads)[0][:, 0], bf.query(reads)[0])
    gb.close()
    gb2.close()


def test_device_api_with_torch_stream(xs, oracle_mod):
    torch = pytest.importorskip("torch")
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=9)
    rng = np.random.default_rng(4)
    reads = _reads(rng, 2000, 21, min_len=150, max_len=151)
    buf = np.frombuffer(b"".join(reads), dtype=np.uint8)
    offs = np.arange(len(reads) + 1, dtype=np.uint64) * 150
    dev = torch.device("cuda", 0)
    d_seqs = torch.from_numpy(buf.copy()).to(dev)
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_hits = torch.empty((len(reads), 100), dtype=torch.int32, device=dev)
    d_nk = torch.empty(len(reads), dtype=torch.int64, device=dev)
    d_tot = torch.empty(101, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    gb.query_device(d_seqs, buf.size, d_offs, len(reads), 1, d_hits, d_nk, d_tot, stream=s.cuda_stream)
    torch.cuda.synchronize()
    want_h, want_n = ob.query(reads)
    assert np.array_equal(d_hits.cpu().numpy().view(np.uint32), want_h)
    assert np.array_equal(d_nk.cpu().numpy().view(np.uint64), want_n)
    tot = d_tot.cpu().numpy().view(np.uint64)
    assert np.array_equal(tot[:100], want_h.sum(axis=0, dtype=np.uint64))
    assert int(tot[100]) == int(want_n.sum())
    gb.close()


@pytest.mark.parametrize("kind", ["cobs", "bloom"])
def test_device_queries_on_mixed_streams(xs, oracle_mod, kind):
    """Queries on one handle from two torch streams and the handle's own host
    API, back to back with no synchronisation in between and growing batches
    (the shared workspace is reallocated mid-sequence): the library orders
    each call after the previous one on the device, so every answer equals
    the oracle's."""
    torch = pytest.importorskip("torch")
    from xspect2_amd.packing import pack_sequences
    rng = np.random.default_rng(77)
    if kind == "cobs":
        ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=5)
        # partitioned COBS on the small bank, in ranges that reuse a 4 MiB workspace
        gb.set_probe_options(cobs_part=2, workspace_mib=4)
        src = seqs
        cols = 100
    else:
        acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
        src = [acgt[rng.integers(0, 4, 60_000)].tobytes()]
        ob = oracle_mod.BloomFilter(np.zeros(20 << 20, dtype=np.uint8), 7, 21)
        ob.build(src)
        gb = xs.Bank.create_bloom(21, 20 << 20, 7)
        gb.set_probe_options(bloom_part=2)
        gb.upload(ob.bits)
        cols = 1
    dev = torch.device("cuda", 0)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    jobs = []
    for i, n in enumerate([200, 3000, 500, 12_000, 800, 20_000]):
        reads = []
        for _ in range(n):
            g = src[int(rng.integers(0, len(src)))]
            st = int(rng.integers(0, max(1, len(g) - 160)))
            reads.append(g[st:st + int(rng.integers(21, 160))])
        reads += _reads(rng, n // 4, 21, min_len=0, max_len=200)
        pr = pack_sequences(reads)
        d_seq = torch.from_numpy(pr.buf[:max(1, int(pr.offsets[-1]))].copy()).to(dev)
        d_off = torch.from_numpy(pr.offsets.astype(np.int64)).to(dev)
        d_hits = torch.empty((pr.n, cols), dtype=torch.int32, device=dev)
        d_nk = torch.empty(pr.n, dtype=torch.int64, device=dev)
        jobs.append((reads, pr, d_seq, d_off, d_hits, d_nk))
    torch.cuda.synchronize()
    host = []
    for i, (reads, pr, d_seq, d_off, d_hits, d_nk) in enumerate(jobs):
        gb.query_device(d_seq, int(pr.offsets[-1]), d_off, pr.n, 1, d_hits, d_nk, None,
                        stream=streams[i % 2].cuda_stream)
        if i == 2:  # the handle's own stream in between, still no sync of the caller's
            host.append((jobs[0][0], gb.query(jobs[0][0])))
    torch.cuda.synchronize()
    host.append((jobs[3][0], gb.query(jobs[3][0])))
    for reads, pr, d_seq, d_off, d_hits, d_nk in jobs:
        want_h, want_n = ob.query(reads)
        assert np.array_equal(d_nk.cpu().numpy().view(np.uint64), want_n)
        assert np.array_equal(d_hits.cpu().numpy().view(np.uint32).reshape(-1), want_h.reshape(-1))
    for reads, (got_h, got_n) in host:
        want_h, want_n = ob.query(reads)
        assert np.array_equal(got_n, want_n) and np.array_equal(got_h.reshape(-1), want_h.reshape(-1))
    gb.close()


@pytest.mark.parametrize("shift", [1, 2, 3])
def test_device_api_unaligned_tight_buffers(xs, oracle_mod, shift):
    """Reads handed over at an unaligned device address, the last read ending
    at the last byte of the buffer, offsets not starting at 0, ragged lengths,
    mixed case and N (window loads stop at the buffer end)."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(shift)
    for D, k, h, sig, bloom in [(100, 21, 7, [30_011], False), (40, 31, 1, [5_003], False), (1, 21, 7, None, True)]:
        if bloom:
            genome = _reads(rng, 3, k, alphabet="ACGTacgtN", min_len=2000, max_len=3000)
            nbytes, K = oracle_mod.BloomFilter.params(9000, 0.01)
            ob = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
            ob.build(genome)
            gb = xs.Bank.create_bloom(k, nbytes, K)
            gb.upload(ob.bits)
            reads = [g[i:i + 150] for g in genome for i in range(0, 1800, 97)]
        else:
            ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, seed=D + shift)
            reads = [s[i:i + int(rng.integers(k - 1, 300))] for s in seqs[:60] for i in (0, 37)]
        reads += _reads(rng, 50, k, alphabet="ACGTacgtNRY", min_len=k - 2, max_len=200)
        lead = 5  # offsets start at 5 inside the handed-over buffer
        body = b"".join(reads)
        raw = np.frombuffer(b"\x00" * shift + b"X" * lead + body, dtype=np.uint8)
        offs = np.zeros(len(reads) + 1, dtype=np.uint64)
        np.cumsum([len(r) for r in reads], out=offs[1:])
        offs += lead
        dev = torch.device("cuda", 0)
        d_all = torch.from_numpy(raw.copy()).to(dev)
        d_seqs = d_all[shift:]  # unaligned base, ends at the last read byte
        assert d_seqs.data_ptr() % 4 == shift % 4 and d_seqs.numel() == lead + len(body)
        d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
        cols = 1 if bloom else D
        d_hits = torch.empty((len(reads), cols), dtype=torch.int32, device=dev)
        d_nk = torch.empty(len(reads), dtype=torch.int64, device=dev)
        gb.query_device(d_seqs, d_seqs.numel(), d_offs, len(reads), 1, d_hits, d_nk, None,
                        stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        want_h, want_n = ob.query(reads)
        assert np.array_equal(d_nk.cpu().numpy().view(np.uint64), want_n)
        assert np.array_equal(d_hits.cpu().numpy().view(np.uint32).reshape(-1), want_h.reshape(-1))
        gb.close()


@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_tiny_k(xs, oracle_mod, k):
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 9, k, 3, [257], seed=k)
    rng = np.random.default_rng(k)
    reads = _reads(rng, 200, k, alphabet="ACGTacgtN", min_len=0, max_len=40)
    for step in (1, 2, 5):
        want_h, want_n = ob.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert np.array_equal(got_n, want_n) and np.array_equal(got_h, want_h)
    gb.close()


def test_mlst_sum_matches_numpy(xs):
    rng = np.random.default_rng(0)
    gb = xs.Bank.create_cobs(21, 1, [101], 50)
    hits = rng.integers(0, 120, (37, 50)).astype(np.uint32)
    owner = np.sort(rng.integers(0, 4, 37)).astype(np.uint32)
    got = gb.mlst_sum(hits, owner, 4, 50)
    want = np.zeros((4, 50), dtype=np.uint64)
    for c in range(37):
        m = hits[c] > 50
        want[owner[c], m] += hits[c, m]
    assert np.array_equal(got, want)
    gb.close()


def _explain(got, want, reads):
    bad = np.flatnonzero((np.asarray(got) != np.asarray(want)).reshape(len(reads), -1).any(axis=1))
    rows = []
    for i in bad[:5]:
        r = reads[i]
        rows.append(f"read {i} len={len(r)} head={r[:30]!r} got={np.asarray(got)[i][:8]} want={np.asarray(want)[i][:8]}")
    return f"{bad.size} rows differ: " + "; ".join(rows)


def test_query_best_matches_hit_matrix(xs, oracle_mod):
    """xs_query_best / xs_best_device == argmax of the hit matrix, ties -> ambiguous."""
    torch = pytest.importorskip("torch")
    for D, k, h, sig in [(100, 21, 7, [20_011]), (3, 31, 1, [997]), (1500, 21, 2, [3_001])]:
        ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, seed=D)
        rng = np.random.default_rng(D)
        reads = [s[o:o + 150] for s in seqs for o in (0, 300)] + _reads(rng, 200, k)
        reads = [r for r in reads if len(r) > 0]
        hits, nk = ob.query(reads)
        hits = hits.reshape(len(reads), D)
        m = hits.max(axis=1)
        ties = (hits == m[:, None]).sum(axis=1)
        want = np.where(ties == 1, hits.argmax(axis=1), 0xFFFFFFFF).astype(np.uint32)
        best, bh, gnk, tot = gb.query_best(reads, want_totals=True)
        assert np.array_equal(best, want) and np.array_equal(bh, m) and np.array_equal(gnk, nk)
        assert np.array_equal(tot[:D], hits.sum(axis=0)) and int(tot[D]) == int(nk.sum())
        dh = torch.from_numpy(hits.astype(np.int32)).cuda()
        db = torch.empty(len(reads), dtype=torch.int32, device="cuda")
        dbh = torch.empty(len(reads), dtype=torch.int32, device="cuda")
        xs.best_device(dh, len(reads), D, db, dbh, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(db.cpu().numpy().view(np.uint32), want)
        assert np.array_equal(dbh.cpu().numpy().view(np.uint32), m)
        gb.close()
    b = xs.Bank.create_bloom(21, 4096, 7)
    best, bh, nk, tot = b.query_best([], want_totals=True)
    assert best.size == 0 and tot.tolist() == [0, 0]
    b.close()


def test_concurrent_handles_from_threads(xs, oracle_mod):
    """The threading contract of include/xspect_hip.h: distinct handles run
    concurrently (ctypes releases the GIL), calls on one handle are serialised
    by its mutex; every result stays bit-exact."""
    from concurrent.futures import ThreadPoolExecutor

    pairs = [_pair(xs, oracle_mod, D, 21, 7, [sig], seed=D) for D, sig in ((50, 9_001), (100, 12_007), (7, 3_001))]
    rng = np.random.default_rng(12)
    batches = [_reads(rng, 400, 21, max_len=250) for _ in range(6)]
    want = {(i, j): pairs[i][0].query(b)[0] for i in range(len(pairs)) for j, b in enumerate(batches)}

    def job(args):
        i, j = args
        return (i, j), pairs[i][1].query(batches[j])[0]

    work = [(i, j) for i in range(len(pairs)) for j in range(len(batches))] * 2  # shared handles too
    with ThreadPoolExecutor(6) as pool:
        for key, got in pool.map(job, work):
            assert np.array_equal(got, want[key]), key
    for _, gb, _, _ in pairs:
        gb.close()


def test_concurrent_large_host_queries_from_threads(xs, oracle_mod):
    """The same contract on the large-call path: batches of 40 k reads go
    through query_host (chunked H2D, the hit rows back on each call's own
    HitSink thread, narrowed and widened) into arrays of the shared host pool
    (bank._HostPool, its lock), four threads over two handles at once;
    every matrix equals the oracle's."""
    from concurrent.futures import ThreadPoolExecutor

    pairs = [_pair(xs, oracle_mod, D, 21, 7, [sig], seed=D + 1) for D, sig in ((100, 12_007), (60, 9_001))]
    rng = np.random.default_rng(13)
    genome = b"".join(pairs[0][2])
    batches = []
    for _ in range(3):  # half random reads, half windows of the first bank's documents
        starts = rng.integers(0, len(genome) - 150, 20_000)
        batches.append(_reads(rng, 20_000, 21, max_len=200) + [genome[o:o + 150] for o in starts])
    want = {(i, j): pairs[i][0].query(b) for i in range(len(pairs)) for j, b in enumerate(batches)}
    assert int(want[(0, 0)][0].sum()) > 0

    def job(args):
        i, j = args
        h, nk = pairs[i][1].query(batches[j])
        ok = np.array_equal(h, want[(i, j)][0]) and np.array_equal(nk, want[(i, j)][1])
        return (i, j), ok, int(h.sum())

    work = [(i, j) for i in range(len(pairs)) for j in range(len(batches))] * 2
    with ThreadPoolExecutor(4) as pool:
        for key, ok, s in pool.map(job, work):
            assert ok, key
            assert s == int(want[key][0].sum())
    for _, gb, _, _ in pairs:
        gb.close()


def test_host_batches_staged_in_chunks(xs, oracle_mod):
    """Host batches larger than one staging chunk (8 MiB first, then 32 MiB)
    are copied and probed chunk by chunk, and their hit rows come back through
    the D2H ring per chunk: hits, k-mer counts, totals and per-read best doc
    must equal the oracle's across every chunk seam, including a read longer
    than a whole staging slot and empty reads at the seams."""
    from xspect2_amd.packing import PackedReads

    ob, gb, _, _ = _pair(xs, oracle_mod, 100, 21, 7, [40_000], seed=5)
    rng = np.random.default_rng(77)
    n = 260_000  # 150-180 bp: ~43 MB, 3 chunks; the second chunk's hit rows (> 64 MB) take the ring
    lens = rng.integers(150, 181, n).astype(np.uint64)
    lens[rng.integers(0, n, 50)] = 0
    offs = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=offs[1:])
    buf = np.frombuffer(b"ACGTN", dtype=np.uint8)[rng.integers(0, 5, int(offs[-1]) + 1)]
    pr = PackedReads(buf, offs)
    want_h, want_n = ob.query_packed(buf, offs)
    got_h, got_n = gb.query(pr)
    assert np.array_equal(got_n, want_n) and np.array_equal(got_h, want_h)
    tot, nk = gb.query_totals(pr)
    assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
    best, bh, bnk, btot = gb.query_best(pr, want_totals=True)
    assert np.array_equal(bh, want_h.max(axis=1)) and np.array_equal(bnk, want_n)
    assert np.array_equal(btot[:100], tot) and int(btot[100]) == nk
    gb.close()

    # one read longer than a staging slot, between short ones, on a small bank
    ob, gb, _, _ = _pair(xs, oracle_mod, 8, 21, 7, [5_000], seed=6)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    seqs = [acgt[rng.integers(0, 4, 200)].tobytes() for _ in range(3)]
    seqs += [acgt[rng.integers(0, 4, 34_000_000)].tobytes()] + seqs
    want_h, want_n = ob.query(seqs)
    got_h, got_n = gb.query(seqs)
    assert np.array_equal(got_n, want_n) and np.array_equal(got_h, want_h)
    tot, nk = gb.query_totals(seqs)
    assert np.array_equal(tot, want_h.sum(axis=0, dtype=np.uint64)) and nk == int(want_n.sum())
    gb.close()


@pytest.mark.parametrize("mode", ["0", "3"])
def test_narrow_host_hits_and_pinned_out(xs, oracle_mod, mode):
    """xs_query_hits: the hit matrix narrowed on the device to uint8 / uint16
    ("auto" picks the narrowest that holds the batch's largest k-mer count)
    equals xs_query's uint32 matrix, on both probe paths, into a fresh or a
    reused pinned buffer (pinned_empty), over several host chunks; a width
    too narrow for the reads is refused."""
    from xspect2_amd import _lib
    from xspect2_amd.bank import pinned_empty
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=4)
    gb.set_probe_options(cobs_part=int(mode))
    rng = np.random.default_rng(4)
    genome = b"".join(seqs)
    reads = [genome[o:o + 150] for o in rng.integers(0, len(genome) - 150, 60_000)] + [b"", b"ACGT"]
    want, want_n = ob.query(reads)
    for dt in (np.uint8, np.uint16, np.uint32, "auto"):
        got, n = gb.query(reads, hit_dtype=dt)
        assert got.dtype == (np.uint8 if dt == "auto" else dt)
        assert np.array_equal(got.astype(np.uint32), want) and np.array_equal(n, want_n)
    out = pinned_empty((len(reads), 100), np.uint8)
    for _ in range(2):
        out[:] = 0xAA
        got, _ = gb.query(reads, hit_dtype=np.uint8, out=out)
        assert got is out and np.array_equal(out.astype(np.uint32), want)
    longr = [genome[:400]]
    with pytest.raises(_lib.XsError):  # 380 k-mers: counts may not fit a byte
        gb.query(longr, hit_dtype=np.uint8)
    got, _ = gb.query(longr, hit_dtype="auto")
    assert got.dtype == np.uint16 and np.array_equal(got, ob.query(longr)[0])
    gb.close()


@pytest.mark.parametrize("mode", ["0", "3"])
def test_device_reads_narrowing_checks_real_counts(xs, oracle_mod, mode):
    """xs_query_hits_device on device-resident reads (a device reader batch's
    form): several chunks, each planned from its own bytes, equal the oracle
    in u8 / u16, totals-only included; a caller's max_len below the longest
    read no longer truncates counts silently: the narrowing kernel flags any
    count wider than hit_bytes and the call fails."""
    import ctypes
    import torch
    from xspect2_amd import _lib
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=6)
    gb.set_probe_options(cobs_part=int(mode))
    rng = np.random.default_rng(6)
    genome = b"".join(seqs)
    reads = [genome[o:o + 150] for o in rng.integers(0, len(genome) - 400, 300_000)] + [genome[:400]]
    want, want_n = ob.query(reads)
    buf = b"".join(reads)
    offs = np.zeros(len(reads) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(r) for r in reads])
    d_seq = torch.from_numpy(np.frombuffer(buf, dtype=np.uint8).copy()).cuda()
    d_off = torch.from_numpy(offs.view(np.int64)).cuda()
    n = len(reads)
    lib = _lib.load()
    for hb, dt, max_len in ((2, np.uint16, 400), (4, np.uint32, 400)):
        hits = np.zeros((n, 100), dtype=dt)
        nk = np.zeros(n, dtype=np.uint64)
        tot = np.zeros(101, dtype=np.uint64)
        rc = lib.xs_query_hits_device(gb.handle, d_seq.data_ptr(), len(buf), d_off.data_ptr(), n, max_len, 1,
                                      hits.ctypes.data, hb, nk.ctypes.data, tot.ctypes.data)
        assert rc == 0, lib.xs_last_error()
        assert np.array_equal(hits.astype(np.uint32), want) and np.array_equal(nk, want_n)
        assert np.array_equal(tot[:100], want.sum(axis=0, dtype=np.uint64)) and int(tot[100]) == int(want_n.sum())
    tot = np.zeros(101, dtype=np.uint64)  # totals only: one chunk
    assert lib.xs_query_hits_device(gb.handle, d_seq.data_ptr(), len(buf), d_off.data_ptr(), n, 400, 1, None, 4,
                                    None, tot.ctypes.data) == 0
    assert np.array_equal(tot[:100], want.sum(axis=0, dtype=np.uint64))
    # the 400-bp read has 380 k-mers: a max_len of 150 claims u8 suffices
    hits = np.zeros((n, 100), dtype=np.uint8)
    rc = lib.xs_query_hits_device(gb.handle, d_seq.data_ptr(), len(buf), d_off.data_ptr(), n, 150, 1,
                                  hits.ctypes.data, 1, None, None)
    assert rc == _lib.XS_ERR_ARG and b"does not fit" in lib.xs_last_error()
    gb.close()


def test_pass_stats_of_the_partitioned_probe(xs, oracle_mod):
    """xs_bank_pass_stats: with profiling on, the partitioned probe's passes
    are timed on the launch stream; their sum is within the probe's own time."""
    ob, gb, seqs, _ = _pair(xs, oracle_mod, 100, 21, 7, [30_011], seed=5)
    gb.set_probe_options(cobs_part=3, workspace_mib=2)  # several workspace ranges
    reads = [s[:150] for s in seqs] * 200
    gb.set_profiling(True)
    gb.probe_stats()
    gb.pass_stats()
    got, _ = gb.query(reads)
    assert np.array_equal(got, ob.query(reads)[0])
    n, tot_ms, _ = gb.probe_stats()
    st = gb.pass_stats()
    assert set(st) == {"prep", "bucket", "lookup", "resolve"}
    assert st["lookup"][1] == st["resolve"][1] == st["bucket"][1] >= 2 and st["prep"][1] >= 1
    assert 0 < sum(ms for ms, _ in st.values()) <= tot_ms * 1.05 + 0.05
    assert gb.pass_stats()["lookup"] == (0.0, 0)  # reset
    gb.set_profiling(False)
    gb.close()


@pytest.mark.parametrize("n_short,n_long,threshold", [(30, 5, 50), (0, 6, 50), (25, 0, 50), (10, 4, 0),
                                                      (3, 3, 1000)])
def test_mlst_query_matches_oracle(xs, oracle_mod, n_short, n_long, threshold):
    """xs_mlst_query against the oracle on a compact bank: direct rows of the
    short sequences; per long sequence the chunk scores > threshold summed per
    allele, the first passing chunk (UINT32_MAX where none) and its score;
    owners with no passing chunk, no short / no long sequences, threshold 0
    (every nonzero count) and a threshold no chunk reaches."""
    D, k, page = 90, 21, 4  # 3 groups of 32 docs
    rng = np.random.default_rng(n_short * 7 + n_long)
    sig = [int(x) for x in rng.integers(3000, 6000, 3)]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, 1, sig, page=page, seed=n_short + 3 * n_long, per_doc=1)
    short = [s[:int(rng.integers(k + 1, len(s) + 1))] for s in seqs[:n_short]]
    chunks, owner = [], []
    for j in range(n_long):
        parts = [seqs[int(rng.integers(0, D))][:int(rng.integers(k + 1, 600))] for _ in range(int(rng.integers(1, 9)))]
        if j == 1:
            parts = [_reads(rng, 1, k, min_len=200, max_len=201)[0]]  # random: nothing passes (usually)
        chunks += parts
        owner += [j] * len(parts)
    n_owners = n_long + 1  # one owner without chunks
    h, sc, first, fs = gb.mlst_query(short, chunks, owner, n_owners, 1, threshold)
    if short:
        want_h, _ = ob.query(short)
        assert np.array_equal(h, want_h)
    else:
        assert h.shape == (0, D)
    rows = ob.query(chunks)[0] if chunks else np.zeros((0, D), np.uint32)
    want_sc = np.zeros((n_owners, D), np.uint64)
    want_first = np.full((n_owners, D), 0xFFFFFFFF, np.uint32)
    want_fs = np.zeros((n_owners, D), np.uint32)
    for c, (o, row) in enumerate(zip(owner, rows)):
        m = row > threshold
        want_sc[o, m] += row[m]
        new = m & (want_first[o] == 0xFFFFFFFF)
        want_first[o, new] = c
        want_fs[o, new] = row[new]
    assert np.array_equal(sc, want_sc) and np.array_equal(first, want_first) and np.array_equal(fs, want_fs)
    gb.close()


def _random_bloom_gather_configs(n=24, seed=20261020):
    rng = np.random.default_rng(seed)
    return [(int(rng.integers(5, 33)), int(rng.integers(64, 3_000_001)), int(rng.integers(1, 17)),
             int(rng.integers(0, 1_000_000))) for _ in range(n)]


@pytest.mark.parametrize("k,nbytes,K,seed", _random_bloom_gather_configs())
def test_bloom_gather_random_configs(xs, oracle_mod, k, nbytes, K, seed):
    """Seeded random rbloom filters through the gather probe (the path
    member-poor input and small filters take: 2 bits first, the rest only for
    k-mers that pass them): k 5-32, 64 B - 3 MB, K 1-16 bit indices, member
    and random reads with lower case, N and IUPAC bytes, steps 1 and 4; the
    device build, hits, counts and totals equal the oracle's."""
    rng = np.random.default_rng(seed)
    genome = _reads(rng, 6, k, alphabet="ACGTacgtN", min_len=k, max_len=4000)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(genome)
    gb = xs.Bank.create_bloom(k, nbytes, K)
    gb.set_probe_options(bloom_part=0)
    gb.build(genome)
    assert np.array_equal(gb.download(), bf.bits), "device-built filter differs"
    reads = _reads(rng, 300, k, alphabet="ACGTacgtNRYKM") + [g[:int(rng.integers(k, len(g) + 1))] for g in genome]
    reads += [b"", b"A" * max(k - 1, 0), genome[0] * 2]
    for step in (1, 4):
        want_h, want_n = bf.query(reads, step=step)
        got_h, got_n = gb.query(reads, step=step)
        assert gb.probe_path() == 0
        assert np.array_equal(got_n, want_n) and np.array_equal(got_h[:, 0], want_h)
        tot, nk = gb.query_totals(reads, step=step)
        assert int(tot[0]) == int(want_h.sum()) and nk == int(want_n.sum())
    gb.close()


def _random_mlst_configs(n=16, seed=20261021):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        page = int(rng.choice([1, 2, 4, 8, 16, 32, 64]))
        G = int(rng.integers(1, 5))
        D = int(rng.integers((G - 1) * 8 * page + 1, G * 8 * page + 1))
        out.append((D, page, G, int(rng.integers(15, 33)), int(rng.integers(1, 4)), int(rng.choice([1, 2, 3])),
                    int(rng.choice([0, 1, 20, 50])), int(rng.integers(0, 1 << 30))))
    return out


# and MLST loci as XspecT trains them (k = 31, one hash, 64-byte pages: the bit-sliced probe)
_VSLICE_MLST = [(400, 64, 1, 31, 1, 1, 50, 11), (900, 64, 2, 31, 1, 2, 20, 12), (1430, 64, 3, 31, 1, 1, 50, 13),
                (2048, 64, 4, 31, 1, 1, 0, 14), (700, 64, 2, 21, 1, 3, 1, 15)]


@pytest.mark.parametrize("D,page,G,k,h,step,threshold,seed", _random_mlst_configs() + _VSLICE_MLST)
def test_mlst_query_random_configs(xs, oracle_mod, D, page, G, k, h, step, threshold, seed):
    """Seeded random compact banks through xs_mlst_query (one MLST locus per
    call, probabilistic_filter_mlst_model.py:192-303): 1-4 groups of pages
    1-64, k 15-32, h 1-3, steps 1-3, thresholds 0 / 1 / 20 / 50; the direct
    rows of short sequences, and per long sequence's chunks the sums of the
    scores over the threshold, the first passing chunk and its score, equal
    the reference's loop restated over the oracle's chunk rows."""
    rng = np.random.default_rng(seed)
    sig = [int(x) for x in rng.integers(700, 4000, G)]
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, page=page, seed=seed % 1000, per_doc=1)
    short = [s[:int(rng.integers(k + 1, len(s) + 1))] for s in seqs[:int(rng.integers(0, 30))]]
    chunks, owner = [], []
    n_long = int(rng.integers(0, 8))
    for j in range(n_long):
        for _ in range(int(rng.integers(1, 9))):
            chunks.append(seqs[int(rng.integers(0, D))][:int(rng.integers(k + 1, 900))])
            owner.append(j)
    n_owners = n_long + 1
    h_, sc, first, fs = gb.mlst_query(short, chunks, owner, n_owners, step, threshold)
    want_h = ob.query(short, step=step)[0] if short else np.zeros((0, D), np.uint32)
    assert np.array_equal(h_, want_h)
    rows = ob.query(chunks, step=step)[0] if chunks else np.zeros((0, D), np.uint32)
    want_sc = np.zeros((n_owners, D), np.uint64)
    want_first = np.full((n_owners, D), 0xFFFFFFFF, np.uint32)
    want_fs = np.zeros((n_owners, D), np.uint32)
    for c, (o, row) in enumerate(zip(owner, rows)):
        m = row > threshold
        want_sc[o, m] += row[m]
        new = m & (want_first[o] == 0xFFFFFFFF)
        want_first[o, new] = c
        want_fs[o, new] = row[new]
    assert np.array_equal(sc, want_sc) and np.array_equal(first, want_first) and np.array_equal(fs, want_fs)
    gb.close()
