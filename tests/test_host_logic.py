"""Host-side logic of the drop-in surface (CPU only, no device calls)."""
from __future__ import annotations

from pathlib import Path

import numpy as np
import pytest

from xspect2_amd import distributed
from xspect2_amd.bank import bloom_parameters, cobs_signature_size
from xspect2_amd.file_io import Record, get_record_iterator, prepare_input_output_paths, write_fasta
from xspect2_amd.packing import pack_fixed, pack_sequences
from xspect2_amd.probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel
from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel, _batches, cobs_result_order
from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
from xspect2_amd.probabilistic_single_filter_model import ProbabilisticSingleFilterModel
from xspect2_amd.util import slugify


def _model(tmp_path, **kw):
    args = dict(k=21, model_display_name="Test Filter", author="John Doe",
                author_email="john.doe@example.com", model_type="Species", base_path=tmp_path)
    args.update(kw)
    return ProbabilisticFilterModel(**args)


def test_slugs_match_reference_tests(tmp_path):
    # tests/test_probabilistic_filter_model.py:125 and test_probabilistic_filter_mlst_model.py:61
    assert _model(tmp_path).slug() == "test-filter-species"
    m = ProbabilisticFilterMlstSchemeModel(21, "MLST (Oxford)", tmp_path, "", "abaumannii")
    assert m.slug() == "abaumannii-mlst-oxford-mlst"
    assert slugify("Acinetobacter") == "acinetobacter"
    assert slugify("A  b--c's 1,000") == "a-b-cs-1000"


def test_constructor_validation(tmp_path):
    with pytest.raises(ValueError):
        _model(tmp_path, k=0)
    with pytest.raises(ValueError):
        _model(tmp_path, model_display_name="")
    with pytest.raises(ValueError):
        _model(tmp_path, model_type="")
    with pytest.raises(ValueError):
        _model(tmp_path, base_path=str(tmp_path))
    m = _model(tmp_path)
    assert (m.fpr, m.num_hashes, m.index) == (0.01, 7, None)
    d = m.to_dict()
    assert d["model_class"] == "ProbabilisticFilterModel" and d["num_hashes"] == 7
    s = ProbabilisticFilterSVMModel(21, "T", None, None, "Species", tmp_path, "rbf", 1.0)
    assert s.to_dict()["kernel"] == "rbf" and s.to_dict()["C"] == 1.0
    g = ProbabilisticSingleFilterModel(21, "T", None, None, "Genus", tmp_path)
    assert g.num_hashes == 1
    mlst = ProbabilisticFilterMlstSchemeModel(21, "S", tmp_path, "u", "org")
    assert (mlst.fpr, mlst.num_hashes, mlst.model_type) == (0.001, 1, "MLST")


def test_count_kmers_known_answer(tmp_path, golden):
    ka = golden("reference_known_answers.json")["salmonella_80bp"]
    m = _model(tmp_path)
    assert m._count_kmers(ka["seq"]) == 60
    assert m._count_kmers(Record("r", ka["seq"])) == 60
    assert m._count_kmers([ka["seq"], ka["seq"]], step=2) == 60
    for step, want in ka["hits_self_by_step"].items():
        assert m._count_kmers(ka["seq"], step=int(step)) == want
    with pytest.raises(ValueError):
        m._count_kmers(42)


def test_input_validation_before_device(tmp_path):
    m = _model(tmp_path)
    with pytest.raises(ValueError, match="Invalid sequence input"):
        m.predict(42)
    with pytest.raises(ValueError, match="longer than k"):
        m.predict([Record("a", "ACGT" * 5)])  # 20 bp <= k
    with pytest.raises(ValueError, match="Bio.Seq"):
        m.calculate_hits(Record("a", "ACGT" * 10))
    with pytest.raises(ValueError, match="longer than k"):
        m.calculate_hits("A" * 21)
    with pytest.raises(NotImplementedError):
        m.predict([Record("a", "A" * 30)], validation=True)
    with pytest.raises(NotImplementedError):  # present, as in the reference (:508), but out of scope
        m.detecting_misclassification({}, [], min_reads=10)


def test_splitter_known_answer_and_oracle(golden, oracle_mod):
    ka = golden("reference_known_answers.json")["splitter"]
    m = ProbabilisticFilterMlstSchemeModel(ka["k"], "Test Filter", Path("."), "", "Test Organism")
    parts = m.sequence_splitter(ka["seq"], ka["allele_len"])
    assert len(parts) == ka["num_parts"]
    rng = np.random.default_rng(0)
    for n in [10_000, 12_345, 999_999, 1_000_000, 1_234_567]:
        seq = "".join(rng.choice(list("ACGT"), n))
        m31 = ProbabilisticFilterMlstSchemeModel(31, "S", Path("."), "", "o")
        assert m31.sequence_splitter(seq, 450) == oracle_mod.sequence_splitter(seq, 450, 31)


def test_has_sufficient_score():
    # tests/test_probabilistic_filter_mlst_model.py:145-177 with Oxford-like sizes
    m = ProbabilisticFilterMlstSchemeModel(21, "S", Path("."), "", "o")
    sizes = [402, 305, 483, 456, 457, 372, 456]
    ok = {"Scores": {"Oxf_cpn60": 265}}
    bad = {"Scores": {"Oxf_cpn60": 100}}
    assert m.has_sufficient_score(ok, sizes)
    assert not m.has_sufficient_score(bad, sizes)
    assert not m.has_sufficient_score({"a": {}}, sizes)


def test_cobs_result_order_is_score_desc_then_index():
    row = np.array([3, 7, 7, 0, 3], dtype=np.uint32)
    assert cobs_result_order(row).tolist() == [1, 2, 0, 4, 3]


def test_packing_and_batches():
    pr = pack_sequences(["ACGT", b"", "GG"])
    assert pr.offsets.tolist() == [0, 4, 4, 6] and pr.buf[:6].tobytes() == b"ACGTGG"
    pf = pack_fixed(np.frombuffer(b"AAAACCCC", dtype=np.uint8).reshape(2, 4))
    assert pf.offsets.tolist() == [0, 4, 8] and pf.n == 2
    import xspect2_amd.probabilistic_filter_model as pfm
    old = pfm.MAX_BATCH_BYTES
    pfm.MAX_BATCH_BYTES = 10
    try:
        assert list(_batches([4, 4, 4, 20, 1])) == [(0, 2), (2, 3), (3, 4), (4, 5)]
    finally:
        pfm.MAX_BATCH_BYTES = old
    assert list(_batches([])) == []


def test_fasta_fastq_io(tmp_path):
    fa = tmp_path / "x.fasta"
    fa.write_text(">r1 desc\nACGT\nAC\n>r2\n\nGG\n")
    recs = list(get_record_iterator(fa))
    assert [(r.id, r.seq) for r in recs] == [("r1", "ACGTAC"), ("r2", "GG")]
    fq = tmp_path / "x.fq"
    fq.write_text("@a 1\nACGT\n+\nIIII\n@b\nGG\n+b\nII\n")
    assert [(r.id, r.seq) for r in get_record_iterator(fq)] == [("a", "ACGT"), ("b", "GG")]
    with pytest.raises(ValueError):
        get_record_iterator(tmp_path / "missing.fasta")
    with pytest.raises(ValueError):
        get_record_iterator(str(fa))
    bad = tmp_path / "x.txt"
    bad.write_text("")
    with pytest.raises(ValueError):
        get_record_iterator(bad)
    write_fasta(recs, tmp_path / "o" / "y.fna", width=3)
    assert [(r.id, r.seq) for r in get_record_iterator(tmp_path / "o" / "y.fna")] == [("r1", "ACGTAC"), ("r2", "GG")]


def test_prepare_input_output_paths(tmp_path):
    (tmp_path / "a.fasta").write_text(">a\nA\n")
    (tmp_path / "b.fq").write_text("@b\nA\n+\nI\n")
    (tmp_path / "c.txt").write_text("")
    ins, fn = prepare_input_output_paths(tmp_path)
    assert [p.name for p in ins] == ["a.fasta", "b.fq"]
    assert fn(1, tmp_path / "out" / "res.json").name == "res_2.json"
    ins, fn = prepare_input_output_paths(tmp_path / "a.fasta")
    assert fn(0, tmp_path / "res.json").name == "res.json"
    with pytest.raises(ValueError):
        prepare_input_output_paths(tmp_path / "nope")


def test_directory_walk_orders_are_the_references(tmp_path):
    """Directory walks happen in the reference's order (iterdir / glob, not
    sorted): species training files (probabilistic_filter_model.py:170-179),
    SVM training genomes (probabilistic_filter_svm_model.py:147-152), the
    MLST locus size (next(glob("*.fasta")), probabilistic_filter_mlst_model.py:
    127-130) and classify inputs (file_io.py:218-221).  The names are chosen
    so that directory order and name order are unlikely to agree."""
    import os
    from xspect2_amd.probabilistic_filter_mlst_model import first_allele_length
    from xspect2_amd.probabilistic_filter_model import training_files
    from xspect2_amd.probabilistic_filter_svm_model import svm_training_files

    rng = np.random.default_rng(3)
    sp = tmp_path / "species"
    sp.mkdir()
    names = [f"{int(x)}.fasta" for x in rng.permutation(40) + 1000] + ["skip.txt", "x.fq"]
    for n in names:
        (sp / n).write_text(">a\nACGT\n")
    (sp / "sub.fasta").mkdir()  # a directory is not a training file
    want = [sp / n for n in os.listdir(sp) if (sp / n).is_file() and n.split(".")[-1] in ("fasta", "fq")]
    assert training_files(sp) == want and len(want) == 41
    svm = tmp_path / "svm"
    for lab in ("470", "28901", "48296"):
        for acc in rng.permutation(6):
            (svm / lab).mkdir(parents=True, exist_ok=True)
            (svm / lab / f"GCF_{acc}.fna").write_text(">a\nACGT\n")
    (svm / "notes.txt").write_text("")
    want = [(svm / lab, svm / lab / f) for lab in os.listdir(svm) if (svm / lab).is_dir()
            for f in os.listdir(svm / lab)]
    assert svm_training_files(svm) == want
    locus = tmp_path / "Oxf_cpn60"
    locus.mkdir()
    for i in rng.permutation(30):
        (locus / f"Allele_ID_{i}.fasta").write_text(f">Oxf_cpn60_{i}\n{'A' * (400 + int(i))}\n>x\nAC\n")
    first = next(n for n in os.listdir(locus) if n.endswith(".fasta"))
    assert first_allele_length(locus) == 400 + int(first.split("_")[-1].split(".")[0])
    ins, _ = prepare_input_output_paths(sp)
    assert ins == [sp / n for e in ("fasta", "fq") for n in os.listdir(sp) if n.endswith("." + e)]


def test_bank_parameter_formulas(oracle_mod):
    for n, h, f in [(4_000_000, 7, 0.01), (600, 1, 0.001)]:
        assert cobs_signature_size(n, h, f) == oracle_mod.signature_size(n, h, f)
    assert bloom_parameters(10_000, 0.01) == oracle_mod.BloomFilter.params(10_000, 0.01)
    with pytest.raises(ValueError):
        bloom_parameters(0, 0.01)


def test_shard_ranges_cover_exactly():
    for n in [0, 1, 7, 100, 1001]:
        for w in [1, 2, 3, 8]:
            rs = [distributed.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


def test_slice_reads():
    pr = pack_sequences(["AAA", "CC", "GGGG", "T"])
    s = distributed.slice_reads(pr, 1, 3)
    assert s.offsets.tolist() == [0, 2, 6] and s.buf[:6].tobytes() == b"CCGGGG"


def test_bench_metric_is_baseline_metric():
    """bench.py reports BASELINE.json's metric verbatim (driver contract)."""
    import importlib.util
    import json
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("bench_mod", root / "bench.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod.METRIC == json.loads((root / "BASELINE.json").read_text())["metric"]


def test_doc_slices_cover_the_bank_in_byte_columns(tmp_path):
    """distributed.doc_slice: contiguous, in order, bounds multiples of 8 (the
    last ends at D), every rank non-empty; too many ranks refused.
    cobs_classic_docs reads the document count of the restated file layout."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
    import oracle
    from xspect2_amd.distributed import cobs_classic_docs, doc_slice
    for D in (1, 8, 9, 13, 100, 128, 129, 2000, 2100):
        R = (D + 7) // 8
        for world in range(1, min(R, 9) + 1):
            sl = [doc_slice(D, r, world) for r in range(world)]
            assert sl[0][0] == 0 and sl[-1][1] == D
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert all(lo < hi and lo % 8 == 0 and (hi % 8 == 0 or hi == D) for lo, hi in sl)
        with pytest.raises(ValueError):
            doc_slice(D, 0, R + 1)
    names = [f"d{i}" for i in range(13)]
    p = tmp_path / "index.cobs_classic"
    p.write_bytes(oracle.cobs_classic_file(names, 21, 7, 11, np.zeros((11, 2), dtype=np.uint8)))
    assert cobs_classic_docs(p) == 13


def test_host_pool_recycles_only_dropped_blocks():
    """Bank.query's result arrays come from recycled host blocks
    (bank._HostPool): a block is reused only once no array or view of it is
    alive, and never beyond the pool's byte cap."""
    import numpy as np
    from xspect2_amd.bank import _HostPool
    p = _HostPool(cap=64 << 20, min_bytes=1 << 20)
    a = p.empty((1000, 4096), np.uint32)            # 16 MB
    view = a[10:20]
    del a
    b = p.empty((1000, 4096), np.uint32)
    assert not np.shares_memory(b, view)            # a view keeps its block busy
    del view
    c = p.empty((1000, 4096), np.uint32)
    assert len(p.blocks) == 2                       # the first block again
    mv = memoryview(b)
    del b
    d = p.empty((1000, 4096), np.uint32)
    assert not np.shares_memory(d, np.asarray(mv)) and not np.shares_memory(d, c)
    e = p.empty((1000, 4096), np.uint32)            # 4 blocks = the 64 MB cap
    f = p.empty((1000, 4096), np.uint32)            # over the cap: a fresh array, not kept
    assert len(p.blocks) == 4 and not any(np.shares_memory(f, x) for x in p.blocks)
    del c, d, e, f, mv
    g = p.empty((2000, 4096), np.uint32)            # 32 MB: free blocks make room for it
    assert g.nbytes == 2000 * 4096 * 4 and sum(x.size for x in p.blocks) <= 64 << 20
    assert p.empty((3, 3), np.uint8).base is None   # small requests: plain arrays
    kept = sum(x.size for x in p.blocks)
    assert p.release() == kept - g.nbytes and [b.size for b in p.blocks] == [g.nbytes]  # g's block stays


def test_host_pool_never_hands_one_block_to_two_threads():
    """Bank.query runs from several threads (the reference's web workers):
    arrays alive at the same time never share a block."""
    import threading
    import numpy as np
    from xspect2_amd.bank import _HostPool
    p = _HostPool(cap=1 << 30, min_bytes=1 << 20)
    bad = []

    def work(t):
        for i in range(200):
            a = p.empty((256, 4096), np.uint8)
            a[:] = t
            if not (a == t).all():
                bad.append((t, i))
            del a

    th = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not bad and sum(b.size for b in p.blocks) <= 1 << 30


def test_save_behind_keeps_order_prints_and_errors(tmp_path, capsys):
    """classify_*'s saves of a directory's results run on one worker thread
    behind the next prediction (classify._SaveBehind): every file is written,
    "Saved result as ..." comes in file order once each save has finished,
    and a failing save raises in the caller."""
    import time
    from xspect2_amd.classify import _SaveBehind

    class Res:
        def __init__(self, text, delay=0.0, fail=False):
            self.text, self.delay, self.fail = text, delay, fail

        def save(self, path):
            time.sleep(self.delay)
            if self.fail:
                raise OSError("disk full")
            path.write_text(self.text)

    s = _SaveBehind()
    for i in range(4):
        s.submit(Res(f"r{i}", delay=0.05 if i % 2 == 0 else 0.0), tmp_path / f"out_{i + 1}.json")
    s.finish()
    assert [(tmp_path / f"out_{i + 1}.json").read_text() for i in range(4)] == ["r0", "r1", "r2", "r3"]
    out = capsys.readouterr().out.splitlines()
    assert out == [f"Saved result as out_{i + 1}.json" for i in range(4)]
    s = _SaveBehind()
    s.submit(Res("x", fail=True), tmp_path / "bad.json")
    with pytest.raises(OSError, match="disk full"):
        s.submit(Res("y"), tmp_path / "next.json")
    s.finish()
    s = _SaveBehind()
    s.submit(Res("x", fail=True), tmp_path / "bad2.json")
    with pytest.raises(OSError, match="disk full"):
        s.finish()
