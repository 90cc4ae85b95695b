"""MatrixResult (columnar results, native JSON writer) against ModelResult.

ModelResult is pinned to the reference class by tests/golden; here the
columnar path must write the very same bytes as ModelResult.save for the same
numbers (json.dumps(indent=4) of to_dict(), result.py:151-202), and agree on
totals, total scores and per-read best docs.  CPU only (host code).
"""
from __future__ import annotations

import numpy as np
import pytest

from xspect2_amd.result import MatrixResult, ModelResult


def _dict_result(slug, ids, labels, hits, nk, step=1, prediction=None, source=None, mask=None):
    docs = np.arange(len(labels)) if mask is None else np.flatnonzero(mask)
    h = {}
    for i, rid in enumerate(ids):
        row = hits[i]
        order = docs[np.argsort(-row[docs].astype(np.int64), kind="stable")]
        h[rid] = {labels[d]: int(row[d]) for d in order}
    n = {rid: int(v) for rid, v in zip(ids, nk)}
    return ModelResult(slug, h, n, step, prediction, source)


CASES = [
    # n, D, max hit, kmers, mask?, prediction, source
    (1, 1, 130, 130, False, None, None),
    (7, 5, 3, 130, False, "470", "reads.fq"),
    (300, 100, 130, 130, False, None, "x.fasta"),
    (50, 12, 40, 97, True, "ambiguous", "y.fq"),
    (20, 3, 0, 11, False, None, None),        # all-zero rows: every doc ties
    (2000, 7, 5, 61, False, "Acinetobacter", "z.fq"),
]


@pytest.mark.parametrize("n,D,hmax,kmers,masked,prediction,source", CASES)
def test_save_is_byte_identical(tmp_path, n, D, hmax, kmers, masked, prediction, source):
    rng = np.random.default_rng(n * 31 + D)
    hits = rng.integers(0, hmax + 1, (n, D)).astype(np.uint32)
    nk = rng.integers(max(kmers // 2, 1), kmers + 1, n).astype(np.uint64)
    hits = np.minimum(hits, nk[:, None]).astype(np.uint32)
    ids = [f"read_{i}" for i in range(n)]
    labels = [f"GCF_{d:09d}" for d in range(D)]
    mask = (rng.random(D) > 0.3).astype(np.uint8) if masked else None
    want = _dict_result("acinetobacter-species", ids, labels, hits, nk, 2, prediction, source, mask)
    got = MatrixResult("acinetobacter-species", ids, labels, hits, nk, 2, prediction, source, mask)
    want.save(tmp_path / "a.json")
    got.save(tmp_path / "b.json")
    assert (tmp_path / "b.json").read_bytes() == (tmp_path / "a.json").read_bytes()
    assert got.get_total_hits() == want.get_total_hits()
    assert got.get_total_scores() == want.get_scores()["total"]
    assert got.to_model_result().to_dict() == want.to_dict()


def test_escaping_duplicates_and_display_labels(tmp_path):
    rng = np.random.default_rng(5)
    ids = ['r"1', "r\\2", "réad3", "r4", "r\t5", "r4"]  # quotes, backslash, non-ASCII, tab, duplicate
    labels = ["470 - baumannii", 'x "quoted"', "ünïcode", "a\nb"]
    hits = rng.integers(0, 20, (len(ids), len(labels))).astype(np.uint32)
    nk = np.full(len(ids), 20, dtype=np.uint64)
    # duplicates: dict semantics keep the first position and the last values
    h, n = {}, {}
    for i, rid in enumerate(ids):
        order = np.argsort(-hits[i].astype(np.int64), kind="stable")
        h[rid] = {labels[d]: int(hits[i, d]) for d in order}
        n[rid] = 20
    want = ModelResult("m", h, n)
    got = MatrixResult("m", ids, labels, hits, nk)
    want.save(tmp_path / "a.json")
    got.save(tmp_path / "b.json")
    assert (tmp_path / "b.json").read_bytes() == (tmp_path / "a.json").read_bytes()


def test_scores_round_like_python():
    """Every (h, n) score string equals repr(round(h / n, 2)) for n up to 300."""
    from xspect2_amd.result import MatrixResult as MR
    import json
    for n in list(range(1, 301)) + [1000, 4096, 99991]:
        hs = range(n + 1) if n <= 300 else range(0, n + 1, max(1, n // 997))
        ids = [f"r{h}" for h in hs]
        hits = np.array(list(hs), dtype=np.uint32)[:, None]
        res = MR("m", ids, ["d"], hits, np.full(len(ids), n, dtype=np.uint64))
        assert res.to_model_result().get_scores()["r0"]["d"] == 0.0
        # through the writer
        import tempfile, os
        with tempfile.TemporaryDirectory() as d:
            res.save(__import__("pathlib").Path(d) / "s.json")
            got = json.loads(open(os.path.join(d, "s.json")).read())["scores"]
            text = open(os.path.join(d, "s.json")).read()
        want = {rid: {"d": round(h / n, 2)} for rid, h in zip(ids, hs)}
        assert {k: v for k, v in got.items() if k != "total"} == want
        for h in list(hs)[:50]:
            assert f'"d": {repr(round(h / n, 2))}' in text


def test_best_and_npz_roundtrip(tmp_path):
    rng = np.random.default_rng(9)
    hits = rng.integers(0, 4, (500, 6)).astype(np.uint32)
    nk = np.full(500, 10, dtype=np.uint64)
    res = MatrixResult("m", [f"r{i}" for i in range(500)], list("abcdef"), hits, nk)
    best, bh = res.best()
    for i in range(500):
        row = hits[i]
        winners = np.flatnonzero(row == row.max())
        assert bh[i] == row.max()
        assert best[i] == (winners[0] if winners.size == 1 else 0xFFFFFFFF)
    res.save_npz(tmp_path / "r.npz")
    back = MatrixResult.load_npz(tmp_path / "r.npz")
    assert back.ids == res.ids and back.labels == res.labels
    assert np.array_equal(back.hits, res.hits) and np.array_equal(back.num_kmers, res.num_kmers)


def test_empty_result_raises_like_reference(tmp_path):
    res = MatrixResult("m", [], ["a"], np.zeros((0, 1), np.uint32), np.zeros(0, np.uint64))
    with pytest.raises(IndexError):
        res.save(tmp_path / "e.json")
    with pytest.raises(ValueError, match="reserved"):
        MatrixResult("m", ["total"], ["a"], np.zeros((1, 1), np.uint32), np.ones(1, np.uint64))


@pytest.mark.parametrize("dtype", [np.uint8, np.uint16])
def test_narrow_hit_matrices_write_the_same_bytes(tmp_path, dtype):
    """A hit matrix narrowed to uint8/uint16 (counts <= k-mers per read) is
    written, summed and converted exactly as the uint32 one."""
    rng = np.random.default_rng(int(np.dtype(dtype).itemsize))
    top = 130 if dtype == np.uint8 else 9000
    nk = rng.integers(top // 2, top + 1, 400).astype(np.uint64)
    hits = np.minimum(rng.integers(0, top + 1, (400, 30)), nk[:, None]).astype(np.uint32)
    ids, labels = [f"r{i}" for i in range(400)], [f"d{j}" for j in range(30)]
    wide = MatrixResult("m", ids, labels, hits, nk, 1, "470", "x.fq")
    narrow = MatrixResult("m", ids, labels, hits.astype(dtype), nk, 1, "470", "x.fq")
    assert narrow.hits.dtype == dtype
    wide.save(tmp_path / "w.json")
    narrow.save(tmp_path / "n.json")
    assert (tmp_path / "n.json").read_bytes() == (tmp_path / "w.json").read_bytes()
    assert narrow.get_total_hits() == wide.get_total_hits()
    assert narrow.to_model_result().to_dict() == wide.to_model_result().to_dict()


@pytest.mark.parametrize("cut", [[0, 37, 120, 200], [0, 0, 150, 200], [0, 200, 200, 200]])
def test_sharded_results_stitch_to_the_whole(tmp_path, cut):
    """Shards of a read-sharded job (set_job_totals: the job's sums, k-mer
    count and first row) write per-read sections for their own reads and the
    job's "total"; merged, they are the whole result's JSON.  A shard without
    reads writes empty sections, as json.dumps does."""
    import json
    from xspect2_amd.distributed import merge_result_shards

    rng = np.random.default_rng(sum(cut))
    n, D = 200, 9
    nk = rng.integers(60, 131, n).astype(np.uint64)
    hits = np.minimum(rng.integers(0, 131, (n, D)), nk[:, None]).astype(np.uint8)
    ids, labels = [f"read_{i}" for i in range(n)], [f"sp{j}" for j in range(D)]
    mask = np.ones(D, np.uint8)
    mask[4] = 0
    whole = MatrixResult("m", ids, labels, hits, nk, 2, "470", "in.fq", mask)
    whole.save(tmp_path / "whole.json")
    paths = []
    for p, (lo, hi) in enumerate(zip(cut, cut[1:])):
        sh = MatrixResult("m", ids[lo:hi], labels, hits[lo:hi], nk[lo:hi], 2, "470", "in.fq", mask)
        sh.set_job_totals(hits.sum(axis=0, dtype=np.uint64), int(nk.sum()), hits[0])
        assert sh.get_total_scores() == whole.get_total_scores()
        sh.save(tmp_path / f"s{p}.json")
        json.loads((tmp_path / f"s{p}.json").read_text())  # every shard is valid JSON
        paths.append(tmp_path / f"s{p}.json")
    assert merge_result_shards(paths) == json.loads((tmp_path / "whole.json").read_text())
    from xspect2_amd.distributed import merge_result_files
    merge_result_files(paths, tmp_path / "merged.json")  # streamed, no parsing: the same bytes
    assert (tmp_path / "merged.json").read_bytes() == (tmp_path / "whole.json").read_bytes()


def test_empty_shard_on_the_dict_path_saves_the_job_total(tmp_path):
    """A shard that takes the dictionary path (equal labels) and holds no
    reads writes empty per-read sections and the job's "total" (ADVICE r3:
    it used to raise IndexError from the local get_total_hits)."""
    import json
    labels = ["a", "a", "b"]
    sh = MatrixResult("m", [], labels, np.zeros((0, 3), np.uint8), np.zeros(0, np.uint64), 1, "470", "in.fq")
    sh.set_job_totals(np.array([10, 20, 30], np.uint64), 100, np.array([1, 2, 3], np.uint32))
    sh.save(tmp_path / "s.json")
    d = json.loads((tmp_path / "s.json").read_text())
    assert d["hits"] == {} and d["num_kmers"] == {}
    assert d["scores"] == {"total": sh.get_total_scores()}
    assert d["prediction"] == "470" and d["input_source"] == "in.fq"
