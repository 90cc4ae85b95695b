"""Pin the CPU oracle before trusting it (CPU only).

* hash layer vs python-xxhash golden vectors (tests/golden/xxh_vectors.json)
* the C restatement vs the independent pure-Python restatement
* the reference tests' own known answers (tests/golden/reference_known_answers.json)
"""
from __future__ import annotations

import math

import numpy as np
import pytest


def test_xxh_golden_vectors(oracle_mod, golden):
    g = golden("xxh_vectors.json")
    assert g["cases"], "empty golden file"
    for case in g["cases"]:
        data = bytes.fromhex(case["hex"])
        for seed, want in enumerate(case["xxh64"]):
            assert oracle_mod.xxh64(data, seed) == int(want), (case["hex"], seed)
        if len(data) <= 240:
            assert oracle_mod.xxh3_64(data) == int(case["xxh3_64"]), case["hex"]


def test_xxh_matches_python_xxhash_random(oracle_mod):
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(3)
    for n in list(range(0, 70)) + [100, 128, 129, 240]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 2**63))
        assert oracle_mod.xxh64(b, s) == xxhash.xxh64_intdigest(b, seed=s)
        assert oracle_mod.xxh3_64(b) == xxhash.xxh3_64_intdigest(b)


@pytest.mark.parametrize("k", [1, 2, 5, 20, 21, 31, 32, 33])
def test_canonical_c_vs_python(oracle_mod, k):
    rng = np.random.default_rng(k)
    for t in range(300):
        alph = "ACGT" if t % 3 else "ACGTNacgtnRYKMSWBDHVXU-"
        s = "".join(rng.choice(list(alph), k))
        assert oracle_mod.canonical_cobs(s.encode()).decode() == oracle_mod.canonical_cobs_py(s)
        assert oracle_mod.canonical_bio(s.encode()).decode() == oracle_mod.canonical_bio_py(s)


def test_canonical_semantics(oracle_mod):
    # reverse complement of AAAC is GTTT; min is AAAC
    assert oracle_mod.canonical_cobs_py("GTTT") == "AAAC"
    assert oracle_mod.canonical_bio_py("GTTT") == "AAAC"
    # case preserved on the genus path, normalised on the COBS path
    assert oracle_mod.canonical_bio_py("gttt") == "aaac"
    assert oracle_mod.canonical_cobs_py("gttt") == "AAAC"
    assert oracle_mod.canonical_cobs_py("ANNT") == "ANNT"


def test_signature_size_formula(oracle_mod):
    for n, h, f in [(4_000_000, 7, 0.01), (500, 1, 0.001), (1, 7, 0.01), (123457, 3, 0.05)]:
        assert oracle_mod.signature_size(n, h, f) == oracle_mod.signature_size_py(n, h, f)
    # ~9.59 rows per term at (h=7, fpr=0.01), ~1000 at (h=1, fpr=0.001)
    assert abs(oracle_mod.signature_size(10**6, 7, 0.01) / 1e6 - 9.594) < 0.01
    assert abs(oracle_mod.signature_size(10**6, 1, 0.001) / 1e6 - 999.5) < 0.5


def test_known_answer_kmer_counts(oracle_mod, golden):
    ka = golden("reference_known_answers.json")["salmonella_80bp"]
    assert oracle_mod.num_kmers(len(ka["seq"]), ka["k"], 1) == ka["num_kmers"]
    for step, want in ka["hits_self_by_step"].items():
        assert oracle_mod.num_kmers(len(ka["seq"]), ka["k"], int(step)) == want
        assert math.ceil((len(ka["seq"]) - ka["k"] + 1) / int(step)) == want


def test_known_answer_splitter(oracle_mod, golden):
    ka = golden("reference_known_answers.json")["splitter"]
    parts = oracle_mod.sequence_splitter(ka["seq"], ka["allele_len"], ka["k"])
    assert len(parts) == ka["num_parts"]
    # every k-mer of the input is in exactly one chunk
    k = ka["k"]
    got = [p[i:i + k] for p in parts for i in range(len(p) - k + 1)]
    want = [ka["seq"][i:i + k] for i in range(len(ka["seq"]) - k + 1)]
    assert got == want


def _small_bank(oracle_mod, D, k, h, seqs_per_doc=2, seed=0, compact_page=None):
    rng = np.random.default_rng(seed)
    docs = []
    for d in range(D):
        for _ in range(seqs_per_doc):
            L = int(rng.integers(k, 400))
            docs.append(("".join(rng.choice(list("ACGT"), L)), d))
    if compact_page is None:
        page, G = (D + 7) // 8, 1
    else:
        page, G = compact_page, (D + 8 * compact_page - 1) // (8 * compact_page)
    sig = [int(rng.integers(50, 3000)) for _ in range(G)]
    bank = oracle_mod.CobsBank.empty(sig, page, D, h, k)
    bank.build([s for s, _ in docs], [d for _, d in docs])
    return bank, docs


@pytest.mark.parametrize("D,k,h,page", [(3, 21, 7, None), (9, 5, 2, None), (20, 31, 1, 1), (17, 16, 3, 1)])
def test_cobs_query_c_vs_python(oracle_mod, D, k, h, page):
    bank, docs = _small_bank(oracle_mod, D, k, h, compact_page=page)
    rng = np.random.default_rng(11)
    queries = [s[: int(rng.integers(k, len(s) + 1))] for s, _ in docs[:6]]
    queries += ["".join(rng.choice(list("ACGTN"), int(rng.integers(k, 200)))) for _ in range(4)]
    queries += ["ACG", ""]  # shorter than k: zero k-mers
    for step in (1, 2, 5):
        hits_c, nk = bank.query(queries, step=step)
        hits_py = bank.query_py(queries, step=step)
        assert np.array_equal(hits_c, hits_py)
        assert [int(x) for x in nk] == [oracle_mod.num_kmers(len(q), k, step) for q in queries]


def test_cobs_self_hits_are_full(oracle_mod):
    """A document's own sequence hits its doc at every position (no false negatives)."""
    bank, docs = _small_bank(oracle_mod, 5, 21, 7, seqs_per_doc=1)
    hits, nk = bank.query([s for s, _ in docs])
    for i, (_, d) in enumerate(docs):
        assert hits[i, d] == nk[i]


def test_bloom_c_vs_python(oracle_mod):
    rng = np.random.default_rng(5)
    seqs = ["".join(rng.choice(list("ACGTacgtN"), int(rng.integers(21, 300)))) for _ in range(8)]
    nbytes, K = oracle_mod.BloomFilter.params(sum(len(s) for s in seqs), 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, 21)
    bf.build(seqs)
    queries = seqs[:4] + ["".join(rng.choice(list("ACGT"), 120)) for _ in range(4)]
    hits, nk = bf.query(queries)
    for q, hv in zip(queries, hits):
        want = sum(bf.contains_py(q[i:i + 21]) for i in range(len(q) - 20))
        assert int(hv) == want
    # inserted k-mers are members
    assert all(int(hits[i]) == int(nk[i]) for i in range(4))


def test_bloom_params_restated(oracle_mod):
    nbytes, K = oracle_mod.BloomFilter.params(1000, 0.01)
    assert K == 7
    assert nbytes == (int(-1000 * math.log(0.01) / math.log(2) ** 2) + 7) // 8


def test_xxh64_seed_terms_equal_the_pinned_hash(oracle_mod):
    """The batched oracle's XXH64 (per-k-mer terms computed once, the seed
    chain per hash) equals xo_xxh64 (pinned to python-xxhash) for every
    length 0..40 and 70 seeds."""
    rng = np.random.default_rng(5)
    L = oracle_mod.lib()
    for n in range(41):
        data = bytes(rng.integers(0, 256, n, dtype=np.uint8))
        for seed in list(range(64)) + [2**32 - 1, 2**32, 2**63, 2**64 - 1, 12345678901, 7]:
            assert L.xo_xxh64_terms_check(data, n, seed) == L.xo_xxh64(data, n, seed), (n, seed)


@pytest.mark.parametrize("D,k,h,page", [(100, 21, 7, None), (3, 21, 7, None), (9, 5, 2, None), (130, 17, 4, None),
                                        (1100, 31, 1, 64), (90, 21, 3, 4), (20, 31, 1, 1), (37, 32, 2, None)])
def test_batched_cobs_query_equals_the_oracle(oracle_mod, D, k, h, page):
    """xo_cobs_query_batched (bench.py's CPU baseline: prefetched rows, seed
    terms computed once, 4 docs per add) gives the scalar oracle's hits and
    counts bit for bit: classic and compact banks, padding docs past D,
    non-ACGT and short reads, steps 1/2/5, threads 1 and 4, and one read of
    more k-mers than a 16-bit counter lane holds (the flush path)."""
    bank, docs = _small_bank(oracle_mod, D, k, h, compact_page=page, seed=D + k)
    rng = np.random.default_rng(D * 3 + k)
    queries = [s[: int(rng.integers(k, len(s) + 1))] for s, _ in docs[:60]]
    queries += ["".join(rng.choice(list("ACGTNacgtRY"), int(rng.integers(0, 300)))) for _ in range(40)]
    queries += ["ACG", "", docs[0][0] * 3]
    long_read = "".join(docs[i % len(docs)][0] for i in range(400))[:70_000 + k]
    queries.append(long_read)  # 70 k sampled k-mers at step 1: past 65535
    buf, offs = oracle_mod.pack(queries)
    for step in (1, 2, 5):
        want_h, want_n = bank.query_packed(buf, offs, step=step)
        for threads in (1, 4):
            got_h, got_n = bank.query_packed_batched(buf, offs, step=step, threads=threads)
            assert np.array_equal(got_n, want_n)
            assert np.array_equal(got_h, want_h), (step, threads, int((got_h != want_h).sum()))
    assert int(want_h[-1].max()) > 0


@pytest.mark.parametrize("nbytes,K,k", [(None, None, 21), (1, 3, 21), (977, 7, 21), (4096, 64, 15),
                                        ((1 << 29) + 12345, 5, 31), (None, None, 240)])
def test_batched_bloom_query_equals_the_oracle(oracle_mod, nbytes, K, k):
    """xo_bloom_query_batched (bench.py's genus CPU baseline: a read's bit
    indices first with Barrett remainders, bytes prefetched ahead) gives the
    scalar oracle's hits and counts bit for bit: sized and overfilled filters,
    one byte, 64 hashes, a filter past 2**32 bits, k 15..240, non-ACGT and short
    reads, steps 1/2/5, threads 1 and 4."""
    rng = np.random.default_rng(k + (nbytes or 0) % 1000)
    seqs = ["".join(rng.choice(list("ACGTacgtN"), int(rng.integers(k, k + 400)))) for _ in range(30)]
    if nbytes is None:
        nbytes, K = oracle_mod.BloomFilter.params(sum(len(s) for s in seqs), 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(seqs)
    queries = seqs[:15] + ["".join(rng.choice(list("ACGTNacgtRY"), int(rng.integers(0, 600)))) for _ in range(40)]
    queries += ["ACG", "", seqs[0] * 3]
    buf, offs = oracle_mod.pack(queries)
    for step in (1, 2, 5):
        want_h, want_n = bf.query_packed(buf, offs, step=step)
        assert int(want_h[:15].min()) > 0 or step > 1
        for threads in (1, 4):
            got_h, got_n = bf.query_packed_batched(buf, offs, step=step, threads=threads)
            assert np.array_equal(got_n, want_n)
            assert np.array_equal(got_h, want_h), (step, threads, int((got_h != want_h).sum()))
    with pytest.raises(ValueError):
        oracle_mod.BloomFilter(np.zeros(0, dtype=np.uint8), 3, k).query_packed_batched(buf, offs)
