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
