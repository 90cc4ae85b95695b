"""filter_genus / filter_species (xspect2_amd.filter_sequences) against the
reference's flow restated on the CPU oracle, byte for byte (GPU).

Reference: ``src/xspect/filter_sequences.py:12-124``: predict the file, save
the classification, ``get_filtered_subsequence_labels(label, threshold)``
(``result.py:92-149``), ``filter_sequences`` (``file_io.py:166-191``: every
record whose id was kept, ``SeqIO.write(..., "fasta")``).  The oracle side
builds its own rbloom filter / COBS bank from the training FASTAs, parses
with the Biopython restatement and writes JSON through ModelResult (pinned to
the reference's result.py); the SVM label comes from the model's own fitted
SVC on the oracle's total scores.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

K = 21


@pytest.fixture
def models(tmp_path, monkeypatch):
    from xspect2_amd.classify import model_dir
    from xspect2_amd.file_io import Record, write_fasta
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
    from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel
    from xspect2_amd.synth import make_genomes

    monkeypatch.setenv("XSPECT_DATA", str(tmp_path / "xd"))
    base = model_dir()
    genomes = [g.tobytes().decode() for g in make_genomes(4, 30_000, seed=8)]
    gfa = tmp_path / "Acinetobacter.fasta"
    write_fasta([Record("g0", genomes[0]), Record("g1", genomes[1])], gfa)
    genus = ProbabilisticSingleFilterModel(K, "Acinetobacter", None, None, "Genus", base)
    genus.fit(gfa, "Acinetobacter")
    genus.save()
    genus.close()
    sdir = tmp_path / "species"
    sdir.mkdir()
    for i in range(4):
        write_fasta([Record(f"c{i}", genomes[i])], sdir / f"{470 + i}.fasta")
    svm = tmp_path / "svm"
    for i in range(4):
        for j in range(2):
            write_fasta([Record("x", genomes[i][j * 7000:j * 7000 + 9000])], svm / f"{470 + i}" / f"acc{i}{j}.fasta")
    species = ProbabilisticFilterSVMModel(K, "Acinetobacter", None, None, "Species", base, "rbf", 1.0)
    species.fit(sdir, svm, svm_step=1)
    species.save()
    species.close()
    return tmp_path, genomes, gfa, sdir


def _reads(tmp_path, genomes, fmt, dup, name="reads", seed=3):
    rng = np.random.default_rng(seed)
    p = tmp_path / f"{name}.{fmt}"
    with open(p, "w") as fh:
        for i in range(400):
            src = genomes[i % 4]
            s = int(rng.integers(0, len(src) - 200))
            seq = src[s:s + int(rng.integers(60, 200))]
            if i % 4 == 0:  # partly foreign: scores between 0 and 1
                seq = seq[:int(rng.integers(21, 60))] + "".join(rng.choice(list("ACGT"), len(seq) - 20))
            rid = f"read{i % 70}" if dup else f"read{i}"
            if fmt == "fq":
                fh.write(f"@{rid} src={i % 4}\n{seq}\n+\n{'I' * len(seq)}\n")
            else:
                fh.write(f">{rid} src={i % 4}\n" + "\n".join(seq[j:j + 60] for j in range(0, len(seq), 60)) + "\n")
    return p


def _oracle_filter(tmp_path, inp, hits_rows, nks, labels, slug, label, threshold, prediction, step):
    """(classification JSON bytes, filtered FASTA bytes or None) of the
    reference's flow from oracle hit rows."""
    import fastx as ofx
    from xspect2_amd.result import ModelResult

    reads = ofx.parse_file(inp)
    titles = ofx.parse_titles(inp)
    hits, nk = {}, {}
    for (rid, _), row, n in zip(reads, hits_rows, nks):
        order = np.argsort(-np.asarray(row, dtype=np.int64), kind="stable")
        hits[rid.decode()] = {labels[i]: int(row[i]) for i in order}
        nk[rid.decode()] = int(n)
    res = ModelResult(slug, hits, nk, step, input_source=inp.name)
    if prediction is not None:
        res.prediction = prediction(res)
    out = tmp_path / "orc"
    out.mkdir(exist_ok=True)
    res.save(out / "cls.json")
    included = set(res.get_filtered_subsequence_labels(label, threshold))
    fasta = None
    if included:
        ofx.write_fasta_bio([(rid, t, s) for (rid, s), t in zip(reads, titles) if rid.decode() in included],
                            out / "f.fasta")
        fasta = (out / "f.fasta").read_bytes()
    return (out / "cls.json").read_bytes(), fasta


@pytest.mark.parametrize("fmt,threshold,dup,step", [("fq", 0.7, False, 1), ("fasta", 0.0, True, 1),
                                                    ("fq", 1.0, False, 2), ("fq", -1, False, 1)])
def test_filter_genus_equals_oracle_flow(models, oracle_mod, fmt, threshold, dup, step):
    import fastx as ofx
    from xspect2_amd.filter_sequences import filter_genus

    tmp_path, genomes, gfa, _ = models
    inp = _reads(tmp_path, genomes, fmt, dup)
    out, cls = tmp_path / "out" / "filtered.fasta", tmp_path / "out" / "genus.json"
    out.parent.mkdir()
    filter_genus("Acinetobacter", inp, out, threshold, cls, step)
    gseqs = [s for _, s in ofx.parse_file(gfa)]
    nbytes, Kh = oracle_mod.BloomFilter.params(sum(map(len, gseqs)) - K + 1, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), Kh, K)
    bf.build(gseqs)
    gh, gn = bf.query([s for _, s in ofx.parse_file(inp)], step=step)
    want_cls, want_fa = _oracle_filter(tmp_path, inp, gh.reshape(-1, 1), gn, ["Acinetobacter"],
                                       "acinetobacter-genus", "Acinetobacter", threshold, None, step)
    assert cls.read_bytes() == want_cls
    assert want_fa is not None and out.read_bytes() == want_fa
    if threshold == -1:
        assert out.read_bytes().count(b">") == len(ofx.parse_file(inp))


@pytest.mark.parametrize("fmt,label,threshold,dup", [("fq", "470", 0.7, False), ("fasta", "471", -1, True),
                                                     ("fq", "473", 0.5, False), ("fq", "470", 1.0, True)])
def test_filter_species_equals_oracle_flow(models, oracle_mod, fmt, label, threshold, dup):
    import fastx as ofx
    from xspect2_amd.classify import species_model_path
    from xspect2_amd.filter_sequences import filter_species
    from xspect2_amd.probabilistic_filter_model import training_files
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    tmp_path, genomes, _, sdir = models
    inp = _reads(tmp_path, genomes, fmt, dup)
    out, cls = tmp_path / "out" / "filtered.fasta", tmp_path / "out" / "species.json"
    out.parent.mkdir()
    filter_species("Acinetobacter", label, inp, out, threshold, cls)
    files = training_files(sdir)
    docs = [s for f in files for _, s in ofx.parse_file(f)]
    D = len(files)
    ob = oracle_mod.CobsBank.empty([oracle_mod.signature_size(max(len(s) - K + 1 for s in docs), 7, 0.01)],
                                   (D + 7) // 8, D, 7, K)
    ob.build(docs, list(range(D)))
    sh, sn = ob.query([s for _, s in ofx.parse_file(inp)], step=1)
    model = ProbabilisticFilterSVMModel.load(species_model_path("Acinetobacter"))
    svc = model._get_svm(None)
    model.close()

    def prediction(res):
        return str(svc.predict([[v for _, v in sorted(res.get_scores()["total"].items())]])[0])

    want_cls, want_fa = _oracle_filter(tmp_path, inp, sh, sn, [f.stem for f in files], "acinetobacter-species",
                                       label, threshold, prediction, 1)
    assert cls.read_bytes() == want_cls
    if want_fa is None:
        assert not out.exists()
    else:
        assert out.read_bytes() == want_fa


def test_filter_genus_directory_input(models, capsys):
    """A directory of inputs: outputs <stem>_<i><suffix> per file in glob
    order (file_io.py prepare_input_output_paths), the reference's messages."""
    from xspect2_amd.filter_sequences import filter_genus

    tmp_path, genomes, _, _ = models
    d = tmp_path / "in"
    d.mkdir()
    _reads(d, genomes, "fq", False, name="a", seed=4)
    _reads(d, genomes, "fasta", False, name="b", seed=5)
    filter_genus("Acinetobacter", d, tmp_path / "o" / "f.fasta", 0.7, tmp_path / "o" / "c.json")
    names = sorted(p.name for p in (tmp_path / "o").iterdir())
    assert names == ["c_1.json", "c_2.json", "f_1.fasta", "f_2.fasta"]
    text = capsys.readouterr().out
    assert "Saved classification results from" in text and "Saved filtered sequences from" in text
