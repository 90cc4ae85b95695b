"""The drop-in model classes on the GPU, checked against the oracle (GPU).

Mirrors the reference's model tests (tests/test_probabilistic_filter_model.py,
test_probabilistic_single_filter_model.py, test_probabilistic_filter_svm_model.py,
test_probabilistic_filter_mlst_model.py) with synthetic genomes in place of
the NCBI / PubMLST downloads, and expected hits from the CPU oracle.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np
import pytest

from xspect2_amd.file_io import Record, get_record_iterator, write_fasta
from xspect2_amd.synth import make_genomes

pytestmark = pytest.mark.gpu

K = 21


@pytest.fixture(scope="module")
def genomes():
    return make_genomes(4, 30_000, seed=11)


@pytest.fixture
def species_dir(tmp_path, genomes):
    d = tmp_path / "species"
    d.mkdir()
    names = ["GCF_000006945.2_ASM694v2_genomic", "GCF_000018445.1_ASM1844v1_genomic",
             "GCF_000069245.1_ASM6924v1_genomic", "GCF_000099999.1_X_genomic"]
    for i, n in enumerate(names):
        g = genomes[i].tobytes().decode()
        # two contigs per species, the second with lower-case and N runs
        write_fasta([Record(f"c{i}a", g[:20_000]), Record(f"c{i}b", g[20_000:25_000].lower() + "NNNN" + g[25_000:])],
                    d / f"{n}.fna", width=80)
    return d


def _oracle_species(oracle_mod, species_dir, k=K, h=7, fpr=0.01):
    from xspect2_amd.probabilistic_filter_model import training_files
    files = training_files(species_dir)  # the reference's iterdir order (doc order of the bank)
    seqs, docs = [], []
    for d, f in enumerate(files):
        for r in get_record_iterator(f):
            seqs.append(r.seq)
            docs.append(d)
    terms = [sum(max(0, len(s) - k + 1) for s, dd in zip(seqs, docs) if dd == d) for d in range(len(files))]
    sig = oracle_mod.signature_size(max(terms), h, fpr)
    ob = oracle_mod.CobsBank.empty([sig], (len(files) + 7) // 8, len(files), h, k)
    ob.build(seqs, docs)
    return ob, [f.stem.split(".")[0] for f in files]


def _expected_hits(ob, names, seqs, step=1, exclude=None):
    h, nk = ob.query(seqs, step=step)
    out = []
    for row in h:
        order = np.argsort(-row.astype(np.int64), kind="stable")
        d = {names[i]: int(row[i]) for i in order}
        if exclude:
            d = {a: b for a, b in d.items() if a not in exclude}
        out.append(d)
    return out, nk


def test_species_fit_predict_save_load(tmp_path, species_dir, genomes, oracle_mod, monkeypatch):
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel

    base = tmp_path / "xspect_data"
    model = ProbabilisticFilterModel(K, "Test Filter", "John Doe", "j@x", "Species", base)
    model.fit(species_dir)
    assert model.display_names["GCF_000006945"] == "GCF_000006945.2_ASM694v2_genomic"
    assert (base / "test-filter-species" / "index.cobs_classic").exists()
    ob, names = _oracle_species(oracle_mod, species_dir)
    assert np.array_equal(model.index.download(), ob.rows), "GPU-built index differs from oracle"

    g0 = genomes[0].tobytes().decode()
    read = g0[1000:1080]  # an 80 bp read of doc 0 -> 60 k-mers (reference :73-93)
    hits = model.calculate_hits(read)
    assert hits["GCF_000006945"] == 60 and list(hits)[0] == "GCF_000006945"
    for step in range(1, 5):
        assert model.calculate_hits(read, step=step)["GCF_000006945"] == -(-60 // step)

    rng = np.random.default_rng(1)
    recs = [Record(f"read_{i}", g0[s:s + 150]) for i, s in enumerate(rng.integers(0, 29_000, 50))]
    recs += [Record("mixed", genomes[1].tobytes().decode()[:5000] + "ACGTN" * 10)]
    res = model.predict(recs, exclude_ids=["GCF_000099999"])
    want, nk = _expected_hits(ob, names, [r.seq for r in recs], exclude=["GCF_000099999"])
    assert list(res.hits) == [r.id for r in recs]
    for r, w in zip(recs, want):
        assert res.hits[r.id] == w and list(res.hits[r.id]) == list(w)
    assert res.num_kmers == {r.id: int(n) for r, n in zip(recs, nk)}

    # Path input, display names, step
    fa = tmp_path / "reads.fasta"
    write_fasta(recs, fa)
    res2 = model.predict(fa, step=3, display_name=True)
    w3, _ = _expected_hits(ob, names, [r.seq for r in recs], step=3)
    key = "GCF_000006945 -GCF_000006945.2_ASM694v2_genomic"
    assert res2.hits["read_0"][key] == w3[0]["GCF_000006945"]

    # FASTQ path streamed in many native batches == the same records in memory
    import xspect2_amd.file_io as fio
    fq = tmp_path / "reads.fq"
    fq.write_text("".join(f"@{r.id} d\n{r.seq}\n+\n{'I' * len(r.seq)}\n" for r in recs))
    monkeypatch.setattr(fio, "DEFAULT_BATCH_TEXT", 1500)
    res4 = model.predict(fq, exclude_ids=["GCF_000099999"])
    assert res4.hits == res.hits and res4.num_kmers == res.num_kmers
    ids, hm, nkm = model.predict_matrix(fq)
    assert ids == [r.id for r in recs] and hm.shape == (len(recs), len(names))
    monkeypatch.undo()

    model.save()
    loaded = ProbabilisticFilterModel.load(base / "test-filter-species.json")
    assert loaded.to_dict() == model.to_dict()
    res3 = loaded.predict(recs)
    assert res3.get_total_hits() == model.predict(recs).get_total_hits()
    with pytest.raises(ValueError):
        loaded.predict([Record("short", "ACGT")])


def test_species_model_same_on_both_probe_paths(tmp_path, species_dir, genomes):
    """predict(), predict_columnar() and the saved JSON are byte-identical whether
    the species bank is probed directly (probe option cobs_part=0) or through
    the partitioned pipeline (=3, forced on this small bank)."""
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel

    model = ProbabilisticFilterModel(K, "Test Filter", "John Doe", "j@x", "Species", tmp_path / "data")
    model.fit(species_dir)
    rng = np.random.default_rng(3)
    src = [g.tobytes().decode() for g in genomes]
    recs = [Record(f"read_{i}", src[i % 4][s:s + int(rng.integers(30, 400))])
            for i, s in enumerate(rng.integers(0, 29_000, 3000))]
    fa = tmp_path / "reads.fasta"
    write_fasta(recs, fa)
    outs = {}
    for mode in ("0", "3"):
        model.index.set_probe_options(cobs_part=int(mode))
        res = model.predict(recs, step=2)
        col = model.predict_columnar(fa)
        path = tmp_path / f"out_{mode}.json"
        col.save(path)
        outs[mode] = (res.hits, res.num_kmers, res.get_scores()["total"], path.read_bytes())
        assert model.index.probe_path() == int(mode == "3")
    assert outs["0"] == outs["3"]


def test_svm_model_vector_and_prediction(tmp_path, species_dir, genomes):
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    svm_dir = tmp_path / "svm"
    for i in range(4):
        for j in range(2):
            g = genomes[i].tobytes().decode()
            write_fasta([Record("x", g[j * 7000:j * 7000 + 9000])], svm_dir / f"label{i}" / f"acc{i}{j}.fasta")
    base = tmp_path / "xspect_data"
    model = ProbabilisticFilterSVMModel(K, "Acinetobacter", None, None, "Species", base, "rbf", 1.0)
    model.fit(species_dir, svm_dir, svm_step=1)
    lines = (base / "acinetobacter-species" / "scores.csv").read_text().splitlines()
    assert lines[0].startswith("file,GCF_000006945,") and lines[0].endswith(",label_id")
    for line in lines[1:]:
        vals = line.split(",")
        lbl = int(vals[-1][-1])
        assert float(vals[1 + lbl]) == 1.0       # own genome scores 1.0 (reference :36-59)
    model.save()
    loaded = ProbabilisticFilterSVMModel.load(base / "acinetobacter-species.json")
    g2 = genomes[2].tobytes().decode()
    res = loaded.predict([Record("q", g2[2000:12_000])], step=5)
    assert res.prediction == "label2"
    vec = ProbabilisticFilterSVMModel.svm_vector(loaded.predict([Record("q", g2[2000:12_000])], step=5))
    assert len(vec) == 4 and vec[2] == 1.0
    # columnar result: same prediction, same JSON bytes as ModelResult.save
    reads = [Record(f"q{i}", g2[s:s + 150]) for i, s in enumerate(range(0, 30_000, 997))]
    fa = tmp_path / "q.fasta"
    write_fasta(reads, fa)
    col = loaded.predict_columnar(fa, exclude_ids=["GCF_000006945"], display_name=True)
    ref = loaded.predict(reads, exclude_ids=["GCF_000006945"], display_name=True)
    assert col.prediction == ref.prediction
    col.input_source = ref.input_source = "q.fasta"
    col.save(tmp_path / "col.json")
    ref.save(tmp_path / "ref.json")
    assert (tmp_path / "col.json").read_bytes() == (tmp_path / "ref.json").read_bytes()


def _mutate(seq: bytes, rate: float, rng) -> bytes:
    a = np.frombuffer(seq, dtype=np.uint8).copy()
    pos = np.flatnonzero(rng.random(a.size) < rate)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    a[pos] = acgt[(np.searchsorted(acgt, a[pos]) + rng.integers(1, 4, pos.size)) % 4]
    return a.tobytes()


@pytest.mark.parametrize("svm_step", [1, 3])
def test_svm_scores_csv_and_label_against_the_oracle(tmp_path, species_dir, genomes, oracle_mod, svm_step):
    """ProbabilisticFilterSVMModel.fit on the GPU writes scores.csv; every row
    equals the row computed on the CPU from the same genomes: the oracle's
    hits of each file's records, the reference's per-record dict (a repeated
    record id keeps its last record, probabilistic_filter_model.py:310),
    totals round(T_d / N, 2) (result.py:57-90) sorted by label and written
    with str() (probabilistic_filter_svm_model.py:144-173), files in the
    reference's iterdir walk order.  The label of a query is then the one an
    SVC fitted on the CPU rows predicts for the oracle's feature vector
    (:208-274)."""
    import fastx  # oracle/fastx.py: the Biopython restatement (test infrastructure)
    from sklearn.svm import SVC
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    rng = np.random.default_rng(17 + svm_step)
    svm_dir = tmp_path / "svm"
    for i in range(4):
        for j in range(3):
            # mutated windows of genome i (and a slice of its neighbour): partial scores
            g = genomes[i].tobytes()
            body = _mutate(g[j * 6000:j * 6000 + 12_000], 0.01 * (j + 1), rng)
            other = genomes[(i + 1) % 4].tobytes()[:2000]
            recs = [Record(f"c{j}", body.decode()), Record("tail", other.decode())]
            if j == 2:  # a repeated record id: the dict keeps the last record
                recs.append(Record("tail", _mutate(other, 0.05, rng).decode()))
            write_fasta(recs, svm_dir / f"label{i}" / f"acc{i}{j}.fasta", width=70)
    base = tmp_path / "xspect_data"
    model = ProbabilisticFilterSVMModel(K, "Acinetobacter", None, None, "Species", base, "rbf", 1.0)
    model.fit(species_dir, svm_dir, svm_step=svm_step)
    got = (base / "acinetobacter-species" / "scores.csv").read_text().split("\n")

    ob, names = _oracle_species(oracle_mod, species_dir)
    want = ["file," + ",".join(sorted(names)) + ",label_id"]
    for folder in svm_dir.iterdir():            # the reference's walk: iterdir, unsorted
        if not folder.is_dir():
            continue
        for f in folder.iterdir():
            if f.suffix[1:] not in ("fasta", "fna", "fa", "ffn", "frn", "fastq", "fq"):
                continue
            recs = fastx.parse_file(f)
            h, nk = ob.query([seq for _, seq in recs], step=svm_step)
            last = {rid: i for i, (rid, _) in enumerate(recs)}          # dict semantics: last record wins
            rows = list(last.values())
            tot = h[rows].sum(axis=0, dtype=np.uint64)
            n_all = int(nk[rows].sum())
            scores = {names[d]: round(int(tot[d]) / n_all, 2) for d in range(len(names))}
            want.append(f"{f.stem}," + ",".join(str(scores[k]) for k in sorted(scores)) + f",{folder.name}")
    assert got == want
    vals = [r.split(",")[1:-1] for r in want[1:]]
    assert any(0 < float(v) < 1 for r in vals for v in r)  # partial scores, not only 0 / 1

    # the label: SVC fitted on the CPU rows, fed the oracle's feature vector of the query
    x = [[float(v) for v in r.split(",")[1:-1]] for r in want[1:]]
    y = [r.split(",")[-1] for r in want[1:]]
    svc = SVC(kernel="rbf", C=1.0).fit(x, y)
    for gi in range(4):
        q = _mutate(genomes[gi].tobytes()[3000:15_000], 0.02, rng)
        h, nk = ob.query([q], step=5)
        feat = [round(int(h[0, d]) / int(nk[0]), 2) for d in np.argsort(names, kind="stable")]
        res = model.predict([Record("q", q.decode())], step=5)
        assert ProbabilisticFilterSVMModel.svm_vector(res) == feat
        assert res.prediction == str(svc.predict([feat])[0])


def test_genus_bloom_model(tmp_path, genomes, oracle_mod):
    from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel

    fa = tmp_path / "concatenated_assembly.fna"
    write_fasta([Record("a", genomes[0].tobytes().decode()), Record("b", genomes[1].tobytes().decode())], fa)
    base = tmp_path / "xspect_data"
    m = ProbabilisticSingleFilterModel(K, "Test Filter", "J", "j@x", "Species", base)
    m.fit(fa, "Acinetobacter baumannii")
    assert m.display_names == {"concatenated_assembly": "Acinetobacter baumannii"}
    total = 2 * genomes.shape[1]
    nbytes, kh = oracle_mod.BloomFilter.params(total - K + 1, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), kh, K)
    bf.build([genomes[0].tobytes(), genomes[1].tobytes()])
    assert np.array_equal(m.bf.download(), bf.bits)
    g0 = genomes[0].tobytes().decode()
    q = g0[500:522]  # 22 bp -> 2 k-mers, both inserted (reference :42-45)
    assert m.calculate_hits(q) == {"concatenated_assembly": 2}
    rng = np.random.default_rng(3)
    reads = [g0[s:s + 150] for s in rng.integers(0, 29_000, 20)] + \
            ["".join(rng.choice(list("ACGTacgtN"), 150)) for _ in range(20)]
    res = m.predict([Record(f"r{i}", s) for i, s in enumerate(reads)])
    want, _ = bf.query(reads)
    assert [res.hits[f"r{i}"]["concatenated_assembly"] for i in range(len(reads))] == want.tolist()
    m.save()
    m2 = ProbabilisticSingleFilterModel.load(base / (m.slug() + ".json"))
    assert m2.to_dict() == m.to_dict()
    assert m2.calculate_hits(q) == {"concatenated_assembly": 2}


def _scheme(tmp_path, rng, loci=3, alleles=40):
    root = tmp_path / "alleles"
    base_seqs = {}
    for li in range(loci):
        base = "".join(rng.choice(list("ACGT"), 450 + 10 * li))
        base_seqs[li] = base
        for a in range(1, alleles + 1):
            s = list(base)
            for p in rng.choice(len(s), size=int(rng.integers(0, 12)), replace=False):
                s[p] = "ACGT"[(("ACGT".index(s[p])) + 1) % 4]
            write_fasta([Record(f"L{li}_{a}", "".join(s))], root / f"Oxf_L{li}" / f"Allele_ID_{a}.fasta")
    return root


def test_mlst_model(tmp_path, oracle_mod):
    from xspect2_amd.probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel

    rng = np.random.default_rng(5)
    root = _scheme(tmp_path, rng)
    base = tmp_path / "xspect_data"
    m = ProbabilisticFilterMlstSchemeModel(K, "MLST (Oxford)", base, "https://example/schemes/1", "abaumannii")
    m.strain_type_resolver = lambda flat, url: "ST" + "-".join(str(v) for v in flat.values())
    m.fit(root, page_size=2)  # 16 alleles per doc group -> 3 groups per locus
    assert len(m.indices) == 3 and all(v == 40 for v in m.loci.values())
    # an allele scores its own k-mer count at its locus (reference :82-99, 401 for cpn60 #4)
    allele = next(get_record_iterator(root / "Oxf_L0" / "Allele_ID_4.fasta")).seq
    res = m.predict(Record("<unknown id>", allele)).hits["test"]
    st = res[0]["Strain type"]["Oxf_L0"]
    assert max(st.values()) == len(allele) - K + 1
    # the compact bank of locus 0 equals the oracle's, and so do its hit rows
    bank0 = m.indices[0]
    assert bank0.info.num_groups == 3
    seqs = {n: next(get_record_iterator(root / "Oxf_L0" / f"{n}.fasta")).seq for n in bank0.doc_names}
    order = bank0.doc_names
    terms = [len(seqs[n]) - K + 1 for n in order]
    assert terms == sorted(terms)
    sig = [oracle_mod.signature_size(max(terms[g * 16:(g + 1) * 16]), 1, 0.001) for g in range(3)]
    ob = oracle_mod.CobsBank.empty(sig, 2, 40, 1, K)
    ob.build([seqs[n] for n in order], list(range(40)))
    assert np.array_equal(bank0.download(), ob.rows)
    q = [seqs[n][10:200] for n in order[:10]] + [allele]
    assert np.array_equal(bank0.query(q)[0], ob.query(q)[0])
    # long path: a 12 kbp contig made of alleles of every locus
    contig = "".join(next(get_record_iterator(root / f"Oxf_L{li}" / "Allele_ID_7.fasta")).seq + "A" * 3000
                     for li in range(3))
    out = m.calculate_hits(contig)
    assert "ST_Name" in out[0]["Strain type"]
    for li in range(3):
        top = out[0]["Strain type"][f"Oxf_L{li}"]
        assert list(top.values())[0] >= 400
    m.save()
    m2 = ProbabilisticFilterMlstSchemeModel.load(base / "abaumannii-mlst-oxford-mlst.json")
    assert m2.loci == m.loci and len(m2.indices) == 3
    m2.strain_type_resolver = m.strain_type_resolver
    assert m2.calculate_hits(contig) == out
    fa = tmp_path / "contigs.fasta"
    write_fasta([Record("c1", contig), Record("c2", allele)], fa)
    mr = m2.predict(fa)
    assert mr.hits["c1"] == out
    with pytest.raises(ValueError):
        m2.predict([Record("x", allele)])


@pytest.mark.parametrize("masked", [True, False])
def test_config1_classify_species_on_an_assembly(tmp_path, species_dir, genomes, oracle_mod, monkeypatch, masked):
    """BASELINE config 1: `xspect classify species` on one assembly FASTA
    (classify.py:70-92 here, reference src/xspect/classify.py:43-92).  The
    assembly is a multi-contig FASTA of one species' genome (lower case, an N
    run, 70-column lines); every contig is one record of thousands of k-mers,
    so each spans many probe units.  The saved JSON's hits, k-mer counts and
    totals must equal the oracle's.

    ``masked=False`` repeats the case with upper-case ACGT only, in the
    training genomes too: its equality does not lean on the unpinned rule for
    lower case and N, which the masked case does."""
    from xspect2_amd import classify
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel

    if not masked:
        species_dir = tmp_path / "species_upper"
        species_dir.mkdir()
        for i, f in enumerate(sorted((tmp_path / "species").iterdir())):
            write_fasta([Record(f"c{i}", genomes[i].tobytes().decode())], species_dir / f.name, width=80)

    root = tmp_path / "xspect-data"
    monkeypatch.setenv("XSPECT_DATA", str(root))
    model = ProbabilisticFilterModel(K, "Acinetobacter", None, None, "Species", root / "models")
    model.fit(species_dir)
    model.save()
    assert classify.species_model_path("Acinetobacter").exists()

    g1 = genomes[1].tobytes().decode()
    contigs = [Record("contig_1 len=12000", g1[:12_000]),
               Record("contig_2", g1[12_000:21_000].lower() + "N" * 40 + g1[21_000:26_000] if masked
                      else g1[12_000:26_000]),
               Record("contig_3", g1[26_000:])]
    fa = tmp_path / "assembly.fna"
    write_fasta(contigs, fa, width=70)
    out = tmp_path / "out" / "result.json"
    from xspect2_amd.bank import Bank
    closed = []
    real_close = Bank.close
    monkeypatch.setattr(Bank, "close", lambda self: (closed.append(self._h is not None), real_close(self))[1])
    classify.classify_species("Acinetobacter", fa, out)
    assert closed and closed[0], "classify_species left its bank open"  # released on return, not at GC
    got = json.loads(out.read_text())

    ob, names = _oracle_species(oracle_mod, species_dir)
    want, nk = _expected_hits(ob, names, [c.seq for c in contigs])
    ids = ["contig_1", "contig_2", "contig_3"]
    assert list(got["hits"]) == ids
    for i, w in zip(ids, want):
        assert got["hits"][i] == w and list(got["hits"][i]) == list(w)
    assert got["num_kmers"] == {i: int(n) for i, n in zip(ids, nk)}
    tot = {d: sum(w[d] for w in want) for d in names}
    assert got["scores"]["total"] == {d: round(tot[d] / int(nk.sum()), 2) for d in tot}
    assert max(tot, key=tot.get) == "GCF_000018445"  # genome 1's species
    assert got["input_source"] == "assembly.fna"


def test_classify_species_directory_saves_behind(tmp_path, species_dir, genomes, monkeypatch, capsys):
    """A directory of inputs through classify_species: each file's result is
    saved on a worker thread while the next file is predicted
    (classify._SaveBehind); the outputs <stem>_<i>.json equal one-file calls
    byte for byte and the "Saved result as" lines come in file order."""
    from xspect2_amd import classify
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel

    root = tmp_path / "xspect-data"
    monkeypatch.setenv("XSPECT_DATA", str(root))
    model = ProbabilisticFilterModel(K, "Acinetobacter", None, None, "Species", root / "models")
    model.fit(species_dir)
    model.save()
    model.close()
    inp = tmp_path / "inputs"
    inp.mkdir()
    for i in range(3):
        g = genomes[i].tobytes().decode()
        write_fasta([Record(f"s{i}_a", g[: 9000 + 1000 * i]), Record(f"s{i}_b", g[12_000:])], inp / f"a{i}.fasta")
    capsys.readouterr()
    classify.classify_species("Acinetobacter", inp, tmp_path / "out" / "res.json")
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("Saved result as")]
    assert lines == [f"Saved result as res_{i + 1}.json" for i in range(3)]
    files, _ = __import__("xspect2_amd.file_io", fromlist=["x"]).prepare_input_output_paths(inp)
    for i, f in enumerate(files):
        one = tmp_path / "one" / f"r{i}.json"
        classify.classify_species("Acinetobacter", f, one)
        assert (tmp_path / "out" / f"res_{i + 1}.json").read_bytes() == one.read_bytes()
