"""Every COBS / rbloom rule that could not be pinned offline, stated once as
an executable spec (CPU).  DESIGN.md §4b lists them; each test here fails if
the implementation stops following the stated rule, and is the one place to
change when the real cobs-reloaded / rbloom become available to pin it.

The GPU side of the same rules: tests/test_gpu_parity.py (the device probes
and builders equal the oracle bit for bit) and
tests/test_gpu_known_answers.py::test_saved_files_follow_the_spec_layouts
(the files the library writes are byte-identical to the spec writers here).
"""
from __future__ import annotations

import math

import numpy as np

K = 21


def test_a1_cobs_canonical_kmer(oracle_mod):
    """A1: canonical = byte-wise min(normalised forward, reverse complement);
    normalisation keeps ACGT, upper-cases acgt, maps every other byte to N;
    the complement swaps A-T, C-G and keeps N."""
    cases = {b"TTTT": b"AAAA", b"acgt": b"ACGT", b"GGGA": b"GGGA", b"TCCC": b"GGGA",
             b"ACGTR": b"ACGTN", b"nnAT": b"ATNN", b"ACGT-": b"ACGTN", b"CCCC": b"CCCC"}
    for kmer, want in cases.items():
        assert oracle_mod.canonical_cobs(kmer) == want, kmer
        assert oracle_mod.canonical_cobs_py(kmer.decode()) == want.decode()


def test_a2_cobs_rows_are_xxh64_mod_s(oracle_mod):
    """A2: a k-mer sets (and is looked up at) row XXH64(canonical, seed=j) mod S
    for j < h, byte d >> 3, bit d & 7 of its doc d."""
    rng = np.random.default_rng(1)
    kmer = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, K)].tobytes()
    S, h, D, d = 1009, 7, 12, 10
    ob = oracle_mod.CobsBank.empty([S], 2, D, h, K)
    ob.build([kmer], [d])
    c = oracle_mod.canonical_cobs(kmer)
    want = np.zeros(S * 2, np.uint8)
    for j in range(h):
        want[(oracle_mod.xxh64(c, j) % S) * 2 + (d >> 3)] |= 1 << (d & 7)
    assert np.array_equal(ob.rows, want)


def test_a3_a4_signature_size_and_compact_groups(oracle_mod):
    """A3: S = ceil(-h n / ln(1 - fpr^(1/h))), n = the largest document's
    k-mer count (positions, duplicates included).  A4: compact banks put
    8 * page_size docs in each group, ordered by (k-mer count, name), each
    group sized by its largest doc (xspect2_amd MLST fit)."""
    for n, h, f in [(4_000_000, 7, 0.01), (570, 1, 0.001), (1, 7, 0.01)]:
        want = math.ceil(-h * n / math.log(1 - f ** (1 / h)))
        assert oracle_mod.signature_size(n, h, f) == want
    from xspect2_amd.bank import cobs_signature_size
    assert cobs_signature_size(4_000_000, 7, 0.01) == 38_371_819  # the config-2 bank: 38.37 M rows
    docs = [(430, "Allele_ID_9"), (421, "Allele_ID_4"), (430, "Allele_ID_10"), (401, "Allele_ID_1")]
    assert [d[1] for d in sorted(docs, key=lambda d: (d[0], d[1]))] == \
        ["Allele_ID_1", "Allele_ID_4", "Allele_ID_10", "Allele_ID_9"]


def test_a5_result_order(oracle_mod):
    """A5: a COBS result lists every doc, score descending, ties by doc index."""
    from xspect2_amd.probabilistic_filter_model import cobs_result_order
    assert cobs_result_order(np.array([0, 5, 5, 2, 0], np.uint32)).tolist() == [1, 2, 3, 0, 4]


def test_b1_b2_rbloom_hash_and_canonical(oracle_mod):
    """B1 (pinned by the reference's own call): hash = xxh3_64_intdigest of the
    canonical k-mer's bytes.  B2: canonical = min(kmer, str(revcomp)) with
    Biopython's IUPAC complement, case preserved (python-xxhash here)."""
    import xxhash
    for kmer in ["ACGTACGTACGTACGTACGTA", "tttttAAAAAcccccGGGGGn", "RYKMSWBDHVNacgtRYKMSW"]:
        c = oracle_mod.canonical_bio_py(kmer)
        assert oracle_mod.canonical_bio(kmer.encode()) == c.encode()
        assert oracle_mod.xxh3_64(c.encode()) == xxhash.xxh3_64_intdigest(c)


def test_b3_rbloom_index_generator(oracle_mod):
    """B3: the K bit indices from the 128-bit LCG seeded with the hash."""
    bf = oracle_mod.BloomFilter(np.zeros(1000, np.uint8), 7, K)
    for hsh in (0, 1, 0xFFFFFFFFFFFFFFFF, 0x0123456789ABCDEF):
        assert bf.indexes(hsh) == oracle_mod.bloom_indexes_py(hsh, 7, 8000)
    # membership: a k-mer is in the filter iff all K bits are set
    kmer = "ACGTTGCAACGTTGCAACGTT"
    bf.build([kmer.encode()])
    c = oracle_mod.canonical_bio_py(kmer).encode()
    idx = oracle_mod.bloom_indexes_py(oracle_mod.xxh3_64(c), 7, 8000)
    set_bits = {i for i in range(8000) if bf.bits[i >> 3] >> (i & 7) & 1}
    assert set_bits == set(idx)


def test_b4_rbloom_sizing(oracle_mod):
    """B4: Bloom(n, fpr): m = floor(-n ln(fpr) / ln(2)^2) bits in ceil(m/8)
    bytes, K = ceil(m / n * ln 2)."""
    from xspect2_amd.bank import bloom_parameters
    for n, f in [(10_000, 0.01), (399_999_980, 0.01), (22, 0.01)]:
        m = int(-n * math.log(f) / math.log(2) ** 2)
        want = ((m + 7) // 8, max(1, math.ceil(m / n * math.log(2))))
        assert bloom_parameters(n, f) == want == oracle_mod.BloomFilter.params(n, f)


def test_c_file_layouts(oracle_mod):
    """A6 / B5: the spec writers produce the layouts the library reads
    (xs_api.cpp read_cobs_header, xs_bank_open): header sizes for a 3-doc
    classic index, a compact index padded to its page, an rbloom file."""
    rows = np.arange(5 * 1, dtype=np.uint8)
    f = oracle_mod.cobs_classic_file(["a", "bb", "c"], K, 7, 5, rows)
    assert f.startswith(b"COBS:CLASSIC_INDEX\x01\x00\x00\x00\x03\x00\x00\x00\x15\x00\x00\x00\x01")
    assert f.endswith(b"a\nbb\nc\nCLASSIC_INDEX" + rows.tobytes())
    cf = oracle_mod.cobs_compact_file(["x", "y"], 31, 1, [3, 4], 8, np.zeros(7 * 8, np.uint8))
    assert (len(cf) - 7 * 8) % 8 == 0 and b"COMPACT_INDEX" in cf
    assert oracle_mod.rbloom_file(7, np.array([1, 2], np.uint8)) == b"\x07" + b"\0" * 7 + b"\x01\x02"
