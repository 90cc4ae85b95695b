"""filter_species / filter_genus building blocks on the CPU: the matrix form of
``get_filter_mask`` against ModelResult's (pinned to the reference's own
``result.py`` by tests/golden/model_result_vectors.json), and
``filter_sequences`` against the Biopython restatement (oracle/fastx.py:
parse, ``record.id in included_ids``, ``SeqIO.write(record, fh, "fasta")``).
Reference: ``src/xspect/filter_sequences.py:12-124``, ``result.py:92-149``,
``file_io.py:166-191``."""
from __future__ import annotations

import numpy as np
import pytest

import fastx as ofx  # test-only checker (oracle/fastx.py)

from xspect2_amd.filter_sequences import filter_sequences
from xspect2_amd.result import MatrixResult, ModelResult

THRESHOLDS = (-1, 0.0, 0.25, 0.5, 0.7, 0.75, 1.0)


def _matrix_of(hits: dict, num_kmers: dict, doc_mask=None) -> MatrixResult:
    ids = list(hits)
    labels = list(next(iter(hits.values())))
    m = np.array([[hits[r][lab] for lab in labels] for r in ids], dtype=np.uint32)
    return MatrixResult("slug", ids, labels, m, np.array([num_kmers[r] for r in ids]), doc_mask=doc_mask)


def test_matrix_masks_equal_the_reference_vectors(golden):
    g = golden("model_result_vectors.json")
    for case in g["cases"]:
        hits = {k: dict(v) for k, v in case["hits"].items()}
        labels = [set(v) for v in hits.values()]
        if any(s != labels[0] for s in labels):
            continue
        mr = _matrix_of(hits, dict(case["num_kmers"]))
        first = next(iter(case["total_hits"]))
        for thr, mask in case["masks"].items():
            assert mr.get_filter_mask(first, float(thr)) == mask
        assert mr.get_filtered_subsequence_labels(first, 0.7) == case["filtered_07"]


@pytest.mark.parametrize("seed", range(6))
def test_matrix_masks_equal_model_result(seed):
    rng = np.random.default_rng(seed)
    n, D = 400, int(rng.integers(1, 9))
    nk = rng.integers(1, 220, n)
    if seed % 2:  # many exact halves: h / n = x.xx5 for n = 200
        nk[:] = 200
    hits = np.minimum(rng.integers(0, 221, (n, D)), nk[:, None]).astype(np.uint32)
    hits[rng.integers(0, n, 30), 0] = nk[rng.integers(0, n, 30)]  # ties with the max
    ids = [f"r{i % 350}" if seed >= 4 else f"r{i}" for i in range(n)]  # seeds 4, 5: repeated ids
    labels = [f"L{d}" for d in range(D)]
    mask = None if seed < 2 or D == 1 else (rng.random(D) < 0.7).astype(np.uint8)
    if mask is not None and not mask.any():
        mask[0] = 1
    mr = MatrixResult("slug", ids, labels, hits.astype(np.uint8 if seed == 3 else np.uint32), nk, doc_mask=mask)
    ref = mr.to_model_result()
    kept = [labels[d] for d in mr.docs.tolist()]
    for lab in kept:
        for thr in THRESHOLDS:
            assert mr.get_filter_mask(lab, thr) == ref.get_filter_mask(lab, thr)
        assert mr.get_filtered_subsequence_labels(lab) == ref.get_filtered_subsequence_labels(lab)


def test_matrix_mask_errors():
    mr = MatrixResult("s", ["a", "b"], ["x", "y"], np.array([[1, 2], [3, 0]], np.uint32), np.array([4, 4]),
                      doc_mask=np.array([1, 0], np.uint8))
    for bad in (-0.5, 1.5, -2):
        with pytest.raises(ValueError):
            mr.get_filter_mask("x", bad)
    with pytest.raises(KeyError):
        mr.get_filter_mask("y", 0.5)  # excluded: not among the reference's labels either
    with pytest.raises(KeyError):
        mr.get_filter_mask("z", 0.5)
    with pytest.raises(KeyError):
        ModelResult("s", {"a": {"x": 1}}, {"a": 4}).get_filter_mask("z", 0.5)
    empty = MatrixResult("s", [], ["x"], np.zeros((0, 1), np.uint32), np.zeros(0, np.uint64))
    with pytest.raises(IndexError):
        empty.get_filter_mask("x", 0.5)
    mis = MatrixResult("s", ["misclassified", "b"], ["x"], np.array([[1], [2]], np.uint32), np.array([4, 4]))
    assert mis.get_filter_mask("x", 0.5) == mis.to_model_result().get_filter_mask("x", 0.5)


def _fastq(rng, ids) -> bytes:
    out = []
    for i, rid in enumerate(ids):
        L = int(rng.integers(30, 200))
        seq = bytes(rng.choice(list(b"ACGT"), L).tolist())
        title = rid + (b" some desc %d" % i if i % 3 else b"")
        out.append(b"@" + title + b"\n" + seq + b"\n+\n" + b"I" * L + b"\n")
    return b"".join(out)


@pytest.mark.parametrize("kind", ["fastq", "fasta"])
def test_filter_sequences_equals_restatement(tmp_path, kind, capsys):
    rng = np.random.default_rng(11)
    ids = [b"r%d" % (i % 900) for i in range(1000)]  # ids 0..99 appear twice
    inp = tmp_path / f"in.{kind}"
    if kind == "fastq":
        inp.write_bytes(_fastq(rng, ids))
    else:
        inp.write_bytes(b"".join(b">%s d%d\n%s\n" % (rid, i, bytes(rng.choice(list(b"ACGTN"), 130).tolist()))
                                 for i, rid in enumerate(ids)))
    wanted = [rid.decode() for rid in ids[::7]]
    out = tmp_path / "out.fasta"
    filter_sequences(inp, out, wanted)
    recs = ofx.parse_file(inp)
    titles = ofx.parse_titles(inp)
    want = [(rid, t, s) for (rid, s), t in zip(recs, titles) if rid.decode() in set(wanted)]
    ofx.write_fasta_bio(want, tmp_path / "want.fasta")
    assert out.read_bytes() == (tmp_path / "want.fasta").read_bytes()
    # no ids: no file, the reference's message
    filter_sequences(inp, tmp_path / "none.fasta", [])
    assert not (tmp_path / "none.fasta").exists()
    assert "No IDs provided, no output file will be created." in capsys.readouterr().out
    # ids that match nothing: the reference has opened (created) the file
    filter_sequences(inp, tmp_path / "empty.fasta", ["nope"])
    assert (tmp_path / "empty.fasta").read_bytes() == b""
    # also where the reference keeps it (src/xspect/file_io.py:166)
    from xspect2_amd import file_io
    file_io.filter_sequences(inp, tmp_path / "out2.fasta", wanted)
    assert (tmp_path / "out2.fasta").read_bytes() == out.read_bytes()
