"""The reference tests' own known answers, pushed through the HIP model classes (GPU).

The reference pins its model classes with three known-answer tests whose
inputs are NCBI / PubMLST downloads (unavailable offline).  The query
sequences and expected numbers are held in
tests/golden/reference_known_answers.json; here each query goes through the
drop-in class on the GPU against a bank built from a FASTA that contains it:

* species (COBS classic): the 80 bp Salmonella read scores 60 for its own
  document and 60/step for steps 1-4, 0 elsewhere
  (reference tests/test_probabilistic_filter_model.py:73-93,149-161);
* genus (rbloom): the 22 bp query scores 2
  (tests/test_probabilistic_single_filter_model.py:42-45,55-56);
* MLST (COBS compact): Oxf_cpn60 Allele_ID_4 (421 bp) scores 401 and is the
  locus' top allele (tests/test_probabilistic_filter_mlst_model.py:82-99).

The other documents are random sequence an order of magnitude smaller than
the one holding the query, so their false-positive rate per k-mer is ~1e-8
and the reference's zeros hold; every hit row is also compared with the CPU
oracle bit for bit.
"""
from __future__ import annotations

import numpy as np
import pytest

from xspect2_amd.file_io import Record, get_record_iterator, write_fasta

pytestmark = pytest.mark.gpu

ACGT = np.frombuffer(b"ACGT", dtype=np.uint8)


def _random(rng, n: int) -> str:
    return ACGT[rng.integers(0, 4, n)].tobytes().decode()


@pytest.fixture
def ka(golden):
    return golden("reference_known_answers.json")


def test_species_salmonella_read(tmp_path, ka, oracle_mod):
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel, training_files

    q = ka["salmonella_80bp"]
    read, k = q["seq"], q["k"]
    rng = np.random.default_rng(6945)
    d = tmp_path / "assemblies"
    d.mkdir()
    genomes = {"GCF_000006945.2_ASM694v2_genomic": _random(rng, 60_000) + read + _random(rng, 40_000),
               "GCF_000018445.1_ASM1844v1_genomic": _random(rng, 10_000),
               "GCF_000069245.1_ASM6924v1_genomic": _random(rng, 10_000)}
    for name, g in genomes.items():
        write_fasta([Record(name.split(".")[0], g)], d / f"{name}.fna", width=80)
    display_names = {"GCF_000006945.2_ASM694v2_genomic": "Salmonella enterica",
                     "GCF_000018445.1_ASM1844v1_genomic": "Acinetobacter baumannii ACICU",
                     "GCF_000069245.1_ASM6924v1_genomic": "Acinetobacter baumannii AYE"}
    model = ProbabilisticFilterModel(k, "Test Filter", "John Doe", "john.doe@example.com", "Species",
                                     tmp_path / "xspect_data")
    model.fit(d, display_names=display_names)
    # reference :97-110: names up to the first ".", in the reference's directory order
    assert model.display_names == {"GCF_000006945": "Salmonella enterica",
                                   "GCF_000018445": "Acinetobacter baumannii ACICU",
                                   "GCF_000069245": "Acinetobacter baumannii AYE"}
    assert list(model.display_names) == [f.stem.split(".")[0] for f in training_files(d)]
    assert model._count_kmers(read) == q["num_kmers"] == 60
    zeros = {"GCF_000069245": 0, "GCF_000018445": 0}
    for step in range(1, 5):
        hits = model.calculate_hits(read, step=step)
        assert hits == {"GCF_000006945": 60 / step, **zeros}          # reference :149-161
        assert hits["GCF_000006945"] == q["hits_self_by_step"][str(step)]
        assert next(iter(hits)) == "GCF_000006945"
    res = model.predict(Record("test", read))                        # reference :73-93
    assert res.get_scores()["total"] == {"GCF_000006945": 1.0, "GCF_000069245": 0.0, "GCF_000018445": 0.0}
    assert res.get_total_hits() == {"GCF_000006945": 60, **zeros}
    assert res.num_kmers == {"test": 60}
    # the same rows from the oracle on the downloaded bank image
    names = model.index.doc_names
    sig = model.index.signature_sizes()
    ob = oracle_mod.CobsBank(model.index.download(), sig, (len(names) + 7) // 8, len(names), 7, k)
    for step in range(1, 5):
        want, nk = ob.query([read.encode()], step=step)
        got, gnk = model.index.query([read], step=step)
        assert np.array_equal(got, want) and np.array_equal(gnk, nk)
    # and the index the GPU built equals the oracle's build from the same files
    seqs, docs = [], []
    for i, f in enumerate(training_files(d)):
        for r in get_record_iterator(f):
            seqs.append(r.seq)
            docs.append(i)
    ob2 = oracle_mod.CobsBank.empty(sig, (len(names) + 7) // 8, len(names), 7, k)
    ob2.build(seqs, docs)
    assert np.array_equal(model.index.download(), ob2.rows)


def test_genus_query(tmp_path, ka, oracle_mod):
    from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel

    q = ka["genus_query"]
    rng = np.random.default_rng(42)
    fa = tmp_path / "concatenated_assembly.fasta"
    write_fasta([Record("a", _random(rng, 30_000) + q["seq"] + _random(rng, 30_000)),
                 Record("b", _random(rng, 20_000))], fa, width=60)
    m = ProbabilisticSingleFilterModel(q["k"], "Test Filter", "John Doe", "john.doe@example.com", "Species",
                                       tmp_path / "xspect_data")
    m.fit(fa, "Acinetobacter baumannii")
    assert m.display_names == {"concatenated_assembly": "Acinetobacter baumannii"}
    hits = m.calculate_hits(q["seq"])
    assert hits == {"concatenated_assembly": q["hits_if_all_present"]} == {"concatenated_assembly": 2}
    m.save()
    loaded = ProbabilisticSingleFilterModel.load(m.base_path / (m.slug() + ".json"))
    assert loaded.to_dict() == m.to_dict()
    assert loaded.calculate_hits(q["seq"]) == {"concatenated_assembly": 2}
    total_length = 30_000 + len(q["seq"]) + 30_000 + 20_000  # Bloom(total_length - k + 1, fpr), :82-88
    nbytes, K = oracle_mod.BloomFilter.params(total_length - q["k"] + 1, 0.01)
    assert (loaded.bf.payload_bytes(), int(loaded.bf.info.num_hashes)) == (nbytes, K)
    bf = oracle_mod.BloomFilter(loaded.bf.download(), K, q["k"])
    want, _ = bf.query([q["seq"].encode()])
    assert int(want[0]) == 2


OXFORD = {"Oxf_cpn60": 265, "Oxf_gdhB": 381, "Oxf_gltA": 241, "Oxf_gpi": 541, "Oxf_gyrB": 352,
          "Oxf_recA": 254, "Oxf_rpoD": 286}


def test_mlst_cpn60_allele4(tmp_path, ka, oracle_mod):
    """A 7-locus scheme with the Oxford allele counts (reference :65-79).
    Oxf_cpn60's Allele_ID_4 is the reference's 421 bp sequence; the other
    alleles of that locus carry 1-8 substitutions, so none holds all 401 of
    its k-mers."""
    from xspect2_amd.probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel

    q = ka["cpn60_allele4"]
    seq, k = q["seq"], q["k"]
    rng = np.random.default_rng(401)
    root = tmp_path / "alleles"
    for locus, count in OXFORD.items():
        base = seq if locus == "Oxf_cpn60" else _random(rng, int(rng.integers(400, 600)))
        for a in range(1, count + 1):
            s = list(base)
            if not (locus == "Oxf_cpn60" and a == 4):
                for p in rng.choice(len(s), size=int(rng.integers(1, 9)), replace=False):
                    s[p] = "ACGT"[("ACGT".index(s[p]) + 1 + int(rng.integers(0, 3))) % 4]
            write_fasta([Record(f"{locus}_{a}", "".join(s))], root / locus / f"Allele_ID_{a}.fasta")
    m = ProbabilisticFilterMlstSchemeModel(k, "MLST (Oxford)", tmp_path / "xspect_data",
                                           "https://rest.pubmlst.org/db/pubmlst_abaumannii_seqdef/schemes/1",
                                           "abaumannii")
    m.strain_type_resolver = lambda flat, url: None  # PubMLST POST: network, out of scope
    m.fit(root)
    assert len(m.indices) == 7 and m.loci == OXFORD
    res = m.predict(Record("<unknown id>", seq)).hits.get("test")[0]
    allele = res.get("Strain type").get("Oxf_cpn60")
    assert allele.get("Allele_ID_4") == q["self_score"] == 401
    assert allele == {"Allele_ID_4": 401}
    # the locus' whole hit row against the oracle on the downloaded compact bank
    li = list(m.loci).index("Oxf_cpn60")
    bank = m.indices[li]
    inf = bank.info
    ob = oracle_mod.CobsBank(bank.download(), bank.signature_sizes(), int(inf.page_size), int(inf.num_docs), 1, k)
    want, nk = ob.query([seq.encode()])
    got, gnk = bank.query([seq])
    assert np.array_equal(got, want) and int(gnk[0]) == 401
    assert int(want[0][bank.doc_names.index("Allele_ID_4")]) == 401


def test_saved_files_follow_the_spec_layouts(tmp_path, oracle_mod):
    """The files the library writes (xs_bank_save) are byte-identical to the
    spec writers of the unverified layouts (oracle.cobs_classic_file,
    cobs_compact_file, rbloom_file), and read back."""
    from xspect2_amd.bank import Bank, bloom_parameters
    from xspect2_amd._lib import XS_BANK_COBS_CLASSIC, XS_BANK_COBS_COMPACT, XS_BANK_RBLOOM
    rng = np.random.default_rng(9)
    seqs = [_random(rng, int(rng.integers(200, 900))) for _ in range(20)]
    names = [f"GCF_{i:09d}" for i in range(10)]
    gb = Bank.create_cobs(21, 7, [3001], 10, names)
    gb.build(seqs, [i % 10 for i in range(20)])
    gb.save(tmp_path / "c.cobs_classic")
    assert (tmp_path / "c.cobs_classic").read_bytes() == oracle_mod.cobs_classic_file(names, 21, 7, 3001,
                                                                                      gb.download())
    gb.close()
    anames = [f"Allele_ID_{i}" for i in range(20)]
    cb = Bank.create_cobs(31, 1, [1500, 2100, 900], 20, anames, page_size=1, compact=True)
    cb.build(seqs, list(range(20)))
    cb.save(tmp_path / "l.cobs_compact")
    assert (tmp_path / "l.cobs_compact").read_bytes() == oracle_mod.cobs_compact_file(anames, 31, 1, [1500, 2100, 900],
                                                                                      1, cb.download())
    cb2 = Bank.open(tmp_path / "l.cobs_compact", XS_BANK_COBS_COMPACT)
    assert cb2.doc_names == anames and np.array_equal(cb2.download(), cb.download())
    cb.close()
    cb2.close()
    nbytes, K = bloom_parameters(5000, 0.01)
    bb = Bank.create_bloom(21, nbytes, K)
    bb.build(seqs)
    bb.save(tmp_path / "filter.bloom")
    assert (tmp_path / "filter.bloom").read_bytes() == oracle_mod.rbloom_file(K, bb.download())
    bb2 = Bank.open(tmp_path / "filter.bloom", XS_BANK_RBLOOM, term_size=21)
    assert np.array_equal(bb2.download(), bb.download())
    bb.close()
    bb2.close()
    assert XS_BANK_COBS_CLASSIC == 0
