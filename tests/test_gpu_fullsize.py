"""BASELINE.json's config 2 at full size on the GPU (1 M x 150 bp reads, a
100-species COBS classic bank of 0.61 GB built on the device from 100 x 4 Mbp
genomes, seed 42: bench.py's species workload), and the genus rbloom filter
over the same genomes (479 MB).

The oracle cannot probe 1.3e10 k-mer x doc pairs in a test's time, so the full
batch is checked through properties that do not depend on its size
(SURVEY.md §8(c)):
* the two independent device probe paths (direct gathers and the partitioned
  bucket -> lookup -> resolve pipeline; for rbloom, gather and partitioned)
  give the same hit matrix, bit for bit;
* per-doc totals equal the hit matrix's column sums and the k-mer total is
  n * 130; every read has 130 k-mers (probabilistic_filter_model.py:462);
* a filter has no false negatives: error-free 150 bp windows of genome d hit
  doc d (species) / the filter (genus) with all 130 k-mers, which pins the
  device-built bank at full size;
* 3,000 reads (the first, the last and a seeded random 1,000) match the C
  oracle probing the downloaded bank image.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, GLEN, N, L, K = 100, 4_000_000, 1_000_000, 150, 21
NK = L - K + 1


@pytest.fixture(scope="module")
def data():
    from xspect2_amd.synth import make_genomes, make_reads
    genomes = make_genomes(D, GLEN, seed=42)
    reads, _ = make_reads(genomes, N, L, seed=42)
    return genomes, reads


@pytest.fixture(scope="module")
def dev_inputs(data):
    torch = pytest.importorskip("torch")
    genomes, reads = data
    dev = torch.device("cuda", 0)
    g = torch.from_numpy(genomes.reshape(-1)).to(dev)
    g_offs = torch.arange(D + 1, dtype=torch.int64, device=dev) * GLEN
    r = torch.from_numpy(reads.reshape(-1)).to(dev)
    r_offs = torch.arange(N + 1, dtype=torch.int64, device=dev) * L
    return torch, dev, g, g_offs, r, r_offs


def _sample_ids():
    rng = np.random.default_rng(7)
    return np.unique(np.concatenate([np.arange(1000), np.arange(N - 1000, N), rng.integers(0, N, 1000)]))


def _windows(genomes, per_doc=20, seed=11):
    """Error-free 150 bp windows, per_doc from each genome, and their doc ids."""
    rng = np.random.default_rng(seed)
    seqs, docs = [], []
    for d in range(D):
        for st in rng.integers(0, GLEN - L + 1, per_doc):
            seqs.append(genomes[d, st:st + L].tobytes())
            docs.append(d)
    return seqs, np.asarray(docs)


def _query(bank, torch, dev, r, r_offs, cols, step=1):
    hits = torch.empty((N, cols), dtype=torch.int32, device=dev)
    nk = torch.empty(N, dtype=torch.int64, device=dev)
    tot = torch.zeros(cols + 1, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev)
    bank.query_device(r, N * L, r_offs, N, step, hits, nk, tot, stream=s.cuda_stream)
    torch.cuda.synchronize(dev)
    return (hits.cpu().numpy().view(np.uint32), nk.cpu().numpy().view(np.uint64),
            tot.cpu().numpy().view(np.uint64), bank.probe_path())


def test_config2_species_full_size(data, dev_inputs, oracle_mod):
    from xspect2_amd import _lib
    from xspect2_amd.bank import Bank, cobs_signature_size
    genomes, reads = data
    torch, dev, g, g_offs, r, r_offs = dev_inputs
    h = 7
    sig = cobs_signature_size(GLEN - K + 1, h, 0.01)
    bank = Bank.create_cobs(K, h, [sig], D, [f"s{i}" for i in range(D)], device=0)
    bank.build_device(g, genomes.size, g_offs, D, torch.arange(D, dtype=torch.int32, device=dev),
                      stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    assert bank.info.device_bytes > 256 << 20  # larger than the Infinity Cache

    bank.set_probe_options(cobs_part=0)
    h0, n0, t0, p0 = _query(bank, torch, dev, r, r_offs, D)
    bank.set_probe_options(cobs_part=1)
    h1, n1, t1, p1 = _query(bank, torch, dev, r, r_offs, D)
    assert p0 == _lib.XS_PATH_GATHER and p1 == _lib.XS_PATH_PARTITIONED
    assert np.array_equal(h0, h1), int((h0 != h1).sum())
    assert np.array_equal(n0, n1) and (n1 == NK).all()
    for t in (t0, t1):
        assert np.array_equal(t[:D], h1.sum(axis=0, dtype=np.uint64)) and int(t[D]) == N * NK
    assert int(h1.max()) <= NK

    # no false negatives at full size: error-free windows of genome d hit doc d with every k-mer
    seqs, docs = _windows(genomes)
    wh, wn = bank.query(seqs)
    assert (wn == NK).all() and (wh[np.arange(len(seqs)), docs] == NK).all()

    # the C oracle on the downloaded bank image, for a sample of the batch
    ob = oracle_mod.CobsBank(bank.download(), [sig], (D + 7) // 8, D, h, K)
    ids = _sample_ids()
    want_h, want_n = ob.query([reads[i].tobytes() for i in ids])
    assert np.array_equal(h1[ids], want_h) and np.array_equal(n1[ids], want_n)
    wo, _ = ob.query(seqs)
    assert np.array_equal(wo, wh)

    # sparse sampling (step 3: 44 k-mers per read, probabilistic_filter_model.py:462) at full
    # size: both paths equal, the counts and totals consistent, the oracle sample equal
    bank.set_probe_options(cobs_part=0)
    s0, m0, u0, _ = _query(bank, torch, dev, r, r_offs, D, step=3)
    bank.set_probe_options(cobs_part=2)
    s1, m1, u1, q1 = _query(bank, torch, dev, r, r_offs, D, step=3)
    assert q1 == _lib.XS_PATH_PARTITIONED and np.array_equal(s0, s1) and np.array_equal(m0, m1)
    assert (m1 == (NK + 2) // 3).all() and np.array_equal(u1[:D], s1.sum(axis=0, dtype=np.uint64))
    want_h, want_n = ob.query([reads[i].tobytes() for i in ids], step=3)
    assert np.array_equal(s1[ids], want_h) and np.array_equal(m1[ids], want_n)
    bank.close()


def test_genus_rbloom_full_size(data, dev_inputs, oracle_mod):
    from xspect2_amd import _lib
    from xspect2_amd.bank import Bank, bloom_parameters
    genomes, reads = data
    torch, dev, g, g_offs, r, r_offs = dev_inputs
    nbytes, nh = bloom_parameters(genomes.size - K + 1, 0.01)  # Bloom(total_length - k + 1, fpr)
    bank = Bank.create_bloom(K, nbytes, nh, device=0)
    bank.build_device(g, genomes.size, g_offs, D, None, stream=torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)

    bank.set_probe_options(bloom_part=0)
    h0, n0, t0, p0 = _query(bank, torch, dev, r, r_offs, 1)
    bank.set_probe_options(bloom_part=2)
    h1, n1, t1, p1 = _query(bank, torch, dev, r, r_offs, 1)
    assert p0 == _lib.XS_PATH_GATHER and p1 == _lib.XS_PATH_PARTITIONED
    assert np.array_equal(h0, h1), int((h0 != h1).sum())
    assert np.array_equal(n0, n1) and (n1 == NK).all()
    for t in (t0, t1):
        assert int(t[0]) == int(h1.sum(dtype=np.uint64)) and int(t[1]) == N * NK

    seqs, _ = _windows(genomes)
    wh, wn = bank.query(seqs)
    assert (wn == NK).all() and (wh[:, 0] == NK).all()

    ob = oracle_mod.BloomFilter(bank.download(), nh, K)
    ids = _sample_ids()
    want_h, want_n = ob.query([reads[i].tobytes() for i in ids])
    assert np.array_equal(h1[ids, 0], want_h) and np.array_equal(n1[ids], want_n)
    bank.close()


def test_config4_mlst_full_size(oracle_mod):
    """Config 4 at full size: 7 loci x 1430 alleles (COBS compact, k = 31,
    h = 1, fpr 0.001, pages of 64 bytes: 3 doc groups per locus, bench.py's
    generator), 1 M error-free 150 bp allele windows.  Per locus, on the
    device: totals = column sums of the 1 M x 1430 hit matrix, 120 k-mers per
    read, and every read taken from allele a of this locus hits allele a with
    all 120 k-mers (no false negatives); 3,000 sampled reads equal the C
    oracle on the downloaded compact bank."""
    torch = pytest.importorskip("torch")
    from xspect2_amd.bank import Bank, cobs_signature_size
    k, loci, n_alleles, page = 31, 7, 1430, 64
    nk = L - k + 1
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    rng = np.random.default_rng(4242)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    li = rng.integers(0, loci, N)
    ai = rng.integers(0, n_alleles, N)
    reads = np.empty((N, L), dtype=np.uint8)
    r = torch.empty(N * L, dtype=torch.uint8, device=dev)
    r_offs = torch.arange(N + 1, dtype=torch.int64, device=dev) * L
    hits = torch.empty((N, n_alleles), dtype=torch.int32, device=dev)
    d_nk = torch.empty(N, dtype=torch.int64, device=dev)
    tot = torch.empty(n_alleles + 1, dtype=torch.int64, device=dev)
    all_alleles, banks = [], []
    for _ in range(loci):
        base = acgt[rng.integers(0, 4, 620)]
        alleles = []
        for _ in range(n_alleles):
            a = base[:int(rng.integers(400, 601))].copy()
            pos = rng.integers(0, a.size, int(rng.integers(0, 12)))
            a[pos] = acgt[(np.searchsorted(acgt, a[pos]) + 1) % 4]
            alleles.append(a)
        alleles.sort(key=lambda a: a.size)  # COBS compact: docs sorted by size
        per = 8 * page
        sig = [cobs_signature_size(max(a.size for a in alleles[g:g + per]) - k + 1, 1, 0.001)
               for g in range(0, n_alleles, per)]
        bank = Bank.create_cobs(k, 1, sig, n_alleles, [f"Allele_ID_{i}" for i in range(n_alleles)],
                                page_size=page, compact=True, device=0)
        buf = np.concatenate(alleles)
        offs = np.zeros(n_alleles + 1, dtype=np.int64)
        offs[1:] = np.cumsum([a.size for a in alleles])
        bank.build_device(torch.from_numpy(buf).to(dev), buf.size, torch.from_numpy(offs).to(dev), n_alleles,
                          torch.arange(n_alleles, dtype=torch.int32, device=dev), stream=s)
        all_alleles.append(alleles)
        banks.append((bank, sig))
    for i in range(N):
        a = all_alleles[li[i]][ai[i]]
        st = int(rng.integers(0, a.size - L + 1))
        reads[i] = a[st:st + L]
    r.copy_(torch.from_numpy(reads.reshape(-1)))
    ids = _sample_ids()
    for locus, (bank, sig) in enumerate(banks):
        bank.query_device(r, N * L, r_offs, N, 1, hits, d_nk, tot, stream=s)
        torch.cuda.synchronize(dev)
        assert bool((d_nk == nk).all())
        assert torch.equal(tot[:n_alleles], hits.sum(dim=0, dtype=torch.int64)) and int(tot[n_alleles]) == N * nk
        mine = torch.from_numpy(np.nonzero(li == locus)[0]).to(dev)
        own = hits[mine, torch.from_numpy(ai[li == locus]).to(dev)]
        assert bool((own == nk).all()), int((own != nk).sum())
        ob = oracle_mod.CobsBank(bank.download(), sig, page, n_alleles, 1, k)
        want_h, want_n = ob.query([reads[i].tobytes() for i in ids])
        got = hits[torch.from_numpy(ids).to(dev)].cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want_h) and np.array_equal(want_n, np.full(ids.size, nk, np.uint64))
        bank.close()


def test_config3_per_gpu_shard(data, dev_inputs, oracle_mod):
    """BASELINE config 3's per-GPU shard: 12.5 M x 150 bp reads (one eighth of
    100 M; seed 42 + rank, here rank 0 -> seed 43) against the replicated
    config-2 bank, in one device call.  The partitioned probe runs it in
    workspace ranges (the bucket blocks of 1.6e9 k-mers reuse one bounded
    workspace); the direct probe gives the same 12.5 M x 100 matrix bit for
    bit, totals equal its column sums, every read has 130 k-mers, and 3,000
    sampled reads equal the C oracle."""
    from xspect2_amd import _lib
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.synth import make_reads
    genomes, _ = data
    torch, dev, g, g_offs, _, _ = dev_inputs
    n = 12_500_000
    reads, _ = make_reads(genomes, n, L, seed=43)
    r = torch.from_numpy(reads.reshape(-1)).to(dev)
    r_offs = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
    h = 7
    sig = cobs_signature_size(GLEN - K + 1, h, 0.01)
    bank = Bank.create_cobs(K, h, [sig], D, [f"s{i}" for i in range(D)], device=0)
    s = torch.cuda.current_stream(dev).cuda_stream
    bank.build_device(g, genomes.size, g_offs, D, torch.arange(D, dtype=torch.int32, device=dev), stream=s)
    out = {}
    for mode in ("0", "1"):
        bank.set_probe_options(cobs_part=int(mode))
        hits = torch.empty((n, D), dtype=torch.int32, device=dev)
        nk = torch.empty(n, dtype=torch.int64, device=dev)
        tot = torch.zeros(D + 1, dtype=torch.int64, device=dev)
        bank.query_device(r, n * L, r_offs, n, 1, hits, nk, tot, stream=s)
        torch.cuda.synchronize(dev)
        out[mode] = (hits, nk, tot, bank.probe_path())
    (h0, n0, t0, p0), (h1, n1, t1, p1) = out["0"], out["1"]
    assert p0 == _lib.XS_PATH_GATHER and p1 == _lib.XS_PATH_PARTITIONED
    assert torch.equal(h0, h1), int((h0 != h1).sum())
    del h0
    assert torch.equal(n0, n1) and bool((n1 == NK).all())
    col = h1.sum(dim=0, dtype=torch.int64)
    for t in (t0, t1):
        assert torch.equal(t[:D], col) and int(t[D]) == n * NK
    assert int(h1.max()) <= NK
    ob = oracle_mod.CobsBank(bank.download(), [sig], (D + 7) // 8, D, h, K)
    rng = np.random.default_rng(8)
    ids = np.unique(np.concatenate([np.arange(1000), np.arange(n - 1000, n), rng.integers(0, n, 1000)]))
    want_h, want_n = ob.query([reads[i].tobytes() for i in ids])
    got = h1[torch.from_numpy(ids).to(dev)].cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want_h) and np.array_equal(want_n, np.full(ids.size, NK, np.uint64))
    bank.close()


def _reference_long_path(model, ob_by_locus, text, limit=False):
    """The reference's long-sequence loop (probabilistic_filter_mlst_model.py:
    236-271), restated over the C oracle's chunk rows: split, keep scores > 50
    per chunk in COBS order, add into an insertion-ordered dict, stable sort
    by -score.  Returns {locus: sorted_counts}."""
    from collections import defaultdict
    out = {}
    for li, (locus, (ob, names)) in enumerate(ob_by_locus.items()):
        parts = model.sequence_splitter(text, model.avg_locus_bp_size[li])
        rows, _ = ob.query([p.encode() for p in parts])
        cobs_results = []
        for row in rows:
            keep = np.flatnonzero(row > 50)
            if keep.size:
                order = keep[np.argsort(-row[keep].astype(np.int64), kind="stable")]
                cobs_results.append({names[d]: int(row[d]) for d in order})
        all_counts = defaultdict(int)
        for res in cobs_results:
            for name, value in res.items():
                all_counts[name] += value
        out[locus] = dict(sorted(all_counts.items(), key=lambda item: -item[1]))
    return out


def test_config4_mlst_long_contigs(oracle_mod):
    """Config 4's long-sequence branch at size: 200 contigs of 10-200 kbp
    (random flanks around alleles of the 7 loci, 1430 alleles each, k = 31),
    through the model's one-call-per-locus path (xs_mlst_query: every chunk
    of every contig probed at once, the > 50 sums and the first passing chunk
    per allele made on the device).  Every contig's per-locus sorted counts,
    keys in order, equal the reference's loop restated over the C oracle's
    chunk rows; the alleles share most k-mers, so equal sums (ties, broken by
    first appearance) are frequent."""
    torch = pytest.importorskip("torch")
    from xspect2_amd.bank import Bank, cobs_signature_size
    from xspect2_amd.probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel
    k, loci, n_alleles, page = 31, 7, 1430, 64
    rng = np.random.default_rng(777)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    model = ProbabilisticFilterMlstSchemeModel(k, "MLST (Oxford)", __import__("pathlib").Path("."), "", "abaumannii")
    oracles, all_alleles = {}, []
    for li in range(loci):
        base = acgt[rng.integers(0, 4, 620)]
        alleles = []
        for _ in range(n_alleles):
            a = base[:int(rng.integers(400, 601))].copy()
            pos = rng.integers(0, a.size, int(rng.integers(0, 12)))
            a[pos] = acgt[(np.searchsorted(acgt, a[pos]) + 1) % 4]
            alleles.append(a)
        alleles.sort(key=lambda a: a.size)
        per = 8 * page
        sig = [cobs_signature_size(max(a.size for a in alleles[g:g + per]) - k + 1, 1, 0.001)
               for g in range(0, n_alleles, per)]
        names = [f"Allele_ID_{i}" for i in range(n_alleles)]
        bank = Bank.create_cobs(k, 1, sig, n_alleles, names, page_size=page, compact=True, device=0)
        bank.build([a.tobytes() for a in alleles], np.arange(n_alleles))
        model.indices.append(bank)
        model.loci[f"Oxf_L{li}"] = n_alleles
        model.avg_locus_bp_size.append(int(alleles[int(rng.integers(0, n_alleles))].size))
        oracles[f"Oxf_L{li}"] = (oracle_mod.CobsBank(bank.download(), sig, page, n_alleles, 1, k), names)
        all_alleles.append(alleles)
    contigs = []
    for c in range(200):
        L = int(rng.integers(10_000, 200_001))
        seq = acgt[rng.integers(0, 4, L)]
        for _ in range(int(rng.integers(0, 4))):  # alleles of random loci inside the flank
            a = all_alleles[int(rng.integers(0, loci))][int(rng.integers(0, n_alleles))]
            at = int(rng.integers(0, L - a.size))
            seq[at:at + a.size] = a
        contigs.append(seq.tobytes().decode())
    rows = model._locus_rows(contigs, 1)
    ties = 0
    for i, text in enumerate(contigs):
        want = _reference_long_path(model, oracles, text)
        for li, locus in enumerate(model.loci):
            got = model._summed_counts(model.indices[li], rows[li][1][i])
            assert list(got.items()) == list(want[locus].items()), (i, locus)
            vals = list(got.values())
            ties += sum(1 for a, b in zip(vals, vals[1:]) if a == b)
    assert ties > 0  # the tie order was exercised
    assert sum(bool(model._summed_counts(model.indices[li], rows[li][1][i])) for i in range(200)
               for li in range(loci)) > 100
    model.close()
