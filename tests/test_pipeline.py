"""Fused genus -> species pipeline (xspect2_amd.pipeline).

CPU: the keep decision equals the reference's round(h / n, 2) >= threshold
(result.py get_filter_mask) on every (h, n).  GPU: one fused pass writes the
same files, byte for byte, as the reference's three-pass flow (genus
predict -> filter by id -> FASTA -> species predict on the FASTA,
main.py:93-160), for FASTA/FASTQ input, several thresholds and repeated ids.
"""
from __future__ import annotations

import numpy as np
import pytest

from xspect2_amd.pipeline import check_threshold, keep_mask


def test_keep_mask_matches_python_round():
    rng = np.random.default_rng(0)
    n = rng.integers(1, 400, 20_000)
    h = (rng.random(20_000) * (n + 1)).astype(np.int64)
    for thr in (0.0, 0.01, 0.5, 0.7, 0.705, 0.99, 1.0):
        want = np.array([round(int(a) / int(b), 2) >= thr for a, b in zip(h, n)])
        assert np.array_equal(keep_mask(h, n, thr), want)
    assert keep_mask(h, n, -1).all()
    for bad in (-0.5, 1.5):
        with pytest.raises(ValueError, match="between 0 and 1"):
            check_threshold(bad)


def _models(tmp_path, k_genus, k_species):
    """A genus Bloom model over 2 synthetic genomes and a 4-species COBS model."""
    from xspect2_amd.file_io import Record, write_fasta
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel
    from xspect2_amd.synth import make_genomes

    genomes = make_genomes(4, 30_000, seed=5)
    gtxt = [g.tobytes().decode() for g in genomes]
    base = tmp_path / "models"
    gfa = tmp_path / "Acinetobacter.fasta"
    write_fasta([Record("g0", gtxt[0]), Record("g1", gtxt[1])], gfa)
    genus = ProbabilisticSingleFilterModel(k_genus, "Acinetobacter", None, None, "Genus", base)
    genus.fit(gfa, "Acinetobacter")
    sdir = tmp_path / "species"
    sdir.mkdir()
    for i in range(4):
        write_fasta([Record(f"c{i}", gtxt[i])], sdir / f"{470 + i}.fasta")
    species = ProbabilisticFilterModel(k_species, "Acinetobacter", None, None, "Species", base)
    species.fit(sdir, display_names={f"{470 + i}": f"Acinetobacter sp{i}" for i in range(4)})
    return genus, species, gtxt


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,threshold,dup", [("fq", 0.7, False), ("fasta", 0.0, False), ("fq", 1.0, False),
                                               ("fq", -1, False), ("fq", 0.7, True)])
def test_fused_pipeline_equals_three_pass(tmp_path, fmt, threshold, dup):
    from xspect2_amd.pipeline import reference_pipeline, run_pipeline

    genus, species, gtxt = _models(tmp_path, 21, 21)

    rng = np.random.default_rng(7)
    recs = []
    for i in range(600):
        src = gtxt[i % 4]
        s = int(rng.integers(0, len(src) - 200))
        seq = src[s:s + int(rng.integers(60, 200))]
        if i % 9 == 0:  # partly foreign reads: scores between 0 and 1
            seq = seq[:40] + "".join(rng.choice(list("ACGT"), len(seq) - 40))
        rid = f"read{i % 50}" if dup else f"read{i}"
        recs.append((rid, f"{rid} source={i % 4}", seq))
    inp = tmp_path / f"reads.{fmt}"
    with open(inp, "w") as fh:
        for rid, desc, seq in recs:
            if fmt == "fq":
                fh.write(f"@{desc}\n{seq}\n+\n{'I' * len(seq)}\n")
            else:
                fh.write(f">{desc}\n{seq}\n")

    import xspect2_amd.file_io as fio
    fio_default = fio.DEFAULT_BATCH_TEXT
    fio.DEFAULT_BATCH_TEXT = 20_000  # many batches
    try:
        got = run_pipeline(genus, species, inp, tmp_path / "fused", threshold=threshold, run_id="r1", log=lambda *a: None)
    finally:
        fio.DEFAULT_BATCH_TEXT = fio_default
    want = reference_pipeline(genus, species, inp, tmp_path / "ref", threshold=threshold, run_id="r1", log=lambda *a: None)
    for key in ("genus", "filtered", "species"):
        assert [p.name for p in got[key]] == [p.name for p in want[key]], key
        for a, b in zip(got[key], want[key]):
            assert a.read_bytes() == b.read_bytes(), (key, a.name)
    if threshold == -1:
        assert got["filtered"] and got["filtered"][0].read_text().count(">") == len(recs)


@pytest.mark.gpu
@pytest.mark.parametrize("short_len,dup", [(25, False), (15, False), (25, True)])
def test_short_read_in_later_batch(tmp_path, short_len, dup):
    """A read too short for a model, in the second batch of a file, fails the
    pipeline with the reference's side effects (main.py:93-160): shorter than
    the genus k -> genus predict raises before anything is written; longer
    than the genus k but not the species k -> the genus JSON and the complete
    filtered FASTA are written (equal to the three-pass flow's), then species
    predict raises.  No partial file is left behind either way."""
    from xspect2_amd.pipeline import reference_pipeline, run_pipeline

    genus, species, gtxt = _models(tmp_path, 21, 31)
    rng = np.random.default_rng(3)
    recs = []
    for i in range(400):
        s = int(rng.integers(0, 29_000))
        L = short_len if i == 300 else int(rng.integers(60, 200))
        rid = f"read{i % 40}" if dup else f"read{i}"
        recs.append((rid, gtxt[i % 4][s:s + L]))
    inp = tmp_path / "reads.fq"
    with open(inp, "w") as fh:
        for rid, seq in recs:
            fh.write(f"@{rid}\n{seq}\n+\n{'I' * len(seq)}\n")
    import xspect2_amd.file_io as fio
    fio_default = fio.DEFAULT_BATCH_TEXT
    fio.DEFAULT_BATCH_TEXT = 20_000  # the short read is in a later batch
    try:
        with pytest.raises(ValueError, match="must be longer than k"):
            run_pipeline(genus, species, inp, tmp_path / "fused", threshold=-1, run_id="r1", log=lambda *a: None)
    finally:
        fio.DEFAULT_BATCH_TEXT = fio_default
    with pytest.raises(ValueError, match="must be longer than k"):
        reference_pipeline(genus, species, inp, tmp_path / "ref", threshold=-1, run_id="r1", log=lambda *a: None)
    got = sorted(p.relative_to(tmp_path / "fused") for p in (tmp_path / "fused").rglob("*") if p.is_file())
    want = sorted(p.relative_to(tmp_path / "ref") for p in (tmp_path / "ref").rglob("*") if p.is_file())
    assert got == want
    for rel in got:
        assert (tmp_path / "fused" / rel).read_bytes() == (tmp_path / "ref" / rel).read_bytes(), rel
    if short_len > 21:
        assert sorted(p.name for p in got) == ["genus_classification_r1.json", "genus_filtered_r1.fasta"]
        filt = (tmp_path / "fused" / "filtered_sequences" / "genus_filtered_r1.fasta").read_text()
        assert filt.count(">") == len(recs)
    else:
        assert got == []


def _oracle_pipeline(oracle_mod, tmp_path, genus, species, inp, threshold, run_id="r1", step=1):
    """The reference's three steps (src/xspect/main.py:93-160,
    filter_sequences.py:71-124) computed from the CPU oracle, independently of
    the HIP path: an rbloom filter and a COBS bank built by the oracle from the
    training FASTAs, Biopython's parse and FASTA write restated
    (oracle/fastx.py), ModelResult (pinned to the reference's result.py) for
    the JSON.  Returns {relative path: bytes} of the files it writes."""
    import fastx as ofx
    from xspect2_amd.probabilistic_filter_model import training_files
    from xspect2_amd.result import ModelResult

    out = {}
    reads = ofx.parse_file(inp)
    titles = ofx.parse_titles(inp)
    # step 1: genus Bloom over the genus FASTA, Bloom(total_length - k + 1, fpr) (:82-88)
    gfa = tmp_path / "Acinetobacter.fasta"
    gseqs = [s for _, s in ofx.parse_file(gfa)]
    nbytes, K = oracle_mod.BloomFilter.params(sum(map(len, gseqs)) - genus.k + 1, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, genus.k)
    bf.build(gseqs)
    gh, gn = bf.query([s for _, s in reads], step=step)
    label = gfa.stem
    hits, nk = {}, {}
    for (rid, _), h, n in zip(reads, gh.tolist(), gn.tolist()):
        hits[rid.decode()] = {label: int(h)}
        nk[rid.decode()] = int(n)
    gres = ModelResult(genus.slug(), hits, nk, step, input_source=inp.name)
    (tmp_path / "orc").mkdir(exist_ok=True)
    gres.save(tmp_path / "orc" / "g.json")
    out[f"genus_classification_{run_id}.json"] = (tmp_path / "orc" / "g.json").read_bytes()
    included = set(gres.get_filtered_subsequence_labels(label, threshold))
    if not included:
        return out
    kept = [(rid, t, s) for (rid, s), t in zip(reads, titles) if rid.decode() in included]
    fname = f"genus_filtered_{run_id}.fasta"
    ofx.write_fasta_bio(kept, tmp_path / "orc" / fname)
    out[f"filtered_sequences/{fname}"] = (tmp_path / "orc" / fname).read_bytes()
    # step 2: species COBS bank over the species FASTAs, docs in the reference's directory order
    files = training_files(tmp_path / "species")
    docs, doc_of = [], []
    for d, f in enumerate(files):
        for _, s in ofx.parse_file(f):
            docs.append(s)
            doc_of.append(d)
    terms = [sum(max(0, len(s) - species.k + 1) for s, o in zip(docs, doc_of) if o == d) for d in range(len(files))]
    D = len(files)
    ob = oracle_mod.CobsBank.empty([oracle_mod.signature_size(max(terms), 7, 0.01)], (D + 7) // 8, D, 7, species.k)
    ob.build(docs, doc_of)
    names = [f.stem.split(".")[0] for f in files]
    freads = ofx.parse_file(tmp_path / "orc" / fname)
    sh, sn = ob.query([s for _, s in freads], step=step)
    hits, nk = {}, {}
    for (rid, _), row, n in zip(freads, sh, sn.tolist()):
        order = np.argsort(-row.astype(np.int64), kind="stable")
        hits[rid.decode()] = {names[i]: int(row[i]) for i in order}
        nk[rid.decode()] = int(n)
    sres = ModelResult(species.slug(), hits, nk, step, input_source=fname)
    sres.save(tmp_path / "orc" / "s.json")
    out[f"species_classification_{run_id}_1.json"] = (tmp_path / "orc" / "s.json").read_bytes()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,threshold,dup", [("fq", 0.0, False), ("fq", 0.7, False), ("fasta", 0.7, True),
                                               ("fq", 1.0, False), ("fasta", -1, False)])
def test_fused_pipeline_equals_oracle(tmp_path, oracle_mod, fmt, threshold, dup):
    """run_pipeline's files against the oracle's restatement of the
    reference's three-pass flow, byte for byte: the genus JSON, the genus keep
    set (thresholds 0, 0.7, 1 and -1, i.e. argmax), the filtered FASTA in
    Bio.SeqIO's layout and the species JSON (main.py:93-187,
    filter_sequences.py:71-124)."""
    from xspect2_amd.pipeline import run_pipeline

    genus, species, gtxt = _models(tmp_path, 21, 21)
    rng = np.random.default_rng(11)
    with open(tmp_path / f"reads.{fmt}", "w") as fh:
        for i in range(500):
            src = gtxt[i % 4]
            s = int(rng.integers(0, len(src) - 200))
            seq = src[s:s + int(rng.integers(60, 200))]
            if i % 5 == 0:  # partly foreign: genus scores between 0 and 1
                seq = seq[:int(rng.integers(21, 60))] + "".join(rng.choice(list("ACGT"), len(seq) - 20))
            rid = f"read{i % 60}" if dup else f"read{i}"
            if fmt == "fq":
                fh.write(f"@{rid} src={i % 4}\n{seq}\n+\n{'I' * len(seq)}\n")
            else:
                fh.write(f">{rid} src={i % 4}\n" + "\n".join(seq[j:j + 70] for j in range(0, len(seq), 70)) + "\n")
    inp = tmp_path / f"reads.{fmt}"
    got = run_pipeline(genus, species, inp, tmp_path / "fused", threshold=threshold, run_id="r1", log=lambda *a: None)
    want = _oracle_pipeline(oracle_mod, tmp_path, genus, species, inp, threshold)
    files = {str(p.relative_to(tmp_path / "fused")): p.read_bytes()
             for key in ("genus", "filtered", "species") for p in got[key]}
    assert sorted(files) == sorted(want)
    for name in want:
        assert files[name] == want[name], name
    if threshold in (0.0, -1):
        assert "species_classification_r1_1.json" in want
