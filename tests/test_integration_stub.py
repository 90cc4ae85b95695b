"""The reference-side ctypes binding (integration/gpu_search.py).

CPU: the stub loads libxspect_hip.so by path and binds only symbols the header
declares; its XsBankInfo mirrors xs_bank_info_t.  GPU: GpuSearch over saved
bank files returns the oracle's hit rows and cobs-style (score, name) lists.
"""
from __future__ import annotations

import ctypes
import importlib.util
import os
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
LIB = ROOT / "xspect2_amd" / "libxspect_hip.so"


def _load_stub():
    if not LIB.exists():
        pytest.skip("libxspect_hip.so not built")
    from xspect2_amd import _lib
    _lib.load()  # same process-wide HIP runtime as the product path
    os.environ["XSPECT_HIP_LIB"] = str(LIB)
    spec = importlib.util.spec_from_file_location("gpu_search", ROOT / "integration" / "gpu_search.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _convert_cobs_result_to_dict(cobs_result) -> dict:
    """Restated consumer: ProbabilisticFilterModel._convert_cobs_result_to_dict
    (src/xspect/models/probabilistic_filter_model.py:393-409)."""
    return {individual_result.doc_name: individual_result.score for individual_result in cobs_result}


def get_cobs_result(cobs_result, kmer_threshold: bool) -> dict:
    """Restated consumer: ProbabilisticFilterMlstSchemeModel.get_cobs_result
    (src/xspect/models/probabilistic_filter_mlst_model.py:362-380)."""
    hits = [result for result in cobs_result if not kmer_threshold or result.score > 50]
    return {result.doc_name: result.score for result in hits}


def test_stub_search_result_shape():
    """search() yields cobs_index.SearchResult-like objects (.doc_name, .score)."""
    mod = _load_stub()
    r = mod.SearchResult("sp3", 60)
    assert (r.doc_name, r.score) == ("sp3", 60)
    assert _convert_cobs_result_to_dict([r, mod.SearchResult("sp1", 0)]) == {"sp3": 60, "sp1": 0}
    assert get_cobs_result([mod.SearchResult("a", 51), mod.SearchResult("b", 50)], True) == {"a": 51}


def test_stub_binds_declared_symbols():
    mod = _load_stub()
    header = (ROOT / "include" / "xspect_hip.h").read_text()
    declared = set(re.findall(r"\b(xs_[a-z_]+)\s*\(", header))
    used = set(re.findall(r"_lib\.(xs_[a-z_]+)", (ROOT / "integration" / "gpu_search.py").read_text()))
    assert used and used <= declared, used - declared
    # xs_bank_info_t: 6 x 32-bit + 7 x 64-bit fields, no padding.
    assert ctypes.sizeof(mod.XsBankInfo) == 6 * 4 + 7 * 8
    assert (mod.COBS_CLASSIC, mod.COBS_COMPACT, mod.RBLOOM) == (0, 1, 2)


def test_integration_doc_matches_stub():
    doc = (ROOT / "INTEGRATION.md").read_text()
    body = (ROOT / "integration" / "gpu_search.py").read_text().split('"""\n', 1)[1]
    assert body in doc, "INTEGRATION.md section 2 is out of sync with integration/gpu_search.py"


@pytest.mark.gpu
def test_stub_search_matches_oracle(oracle_mod, tmp_path):
    mod = _load_stub()
    from xspect2_amd import bank as xs

    rng = np.random.default_rng(11)
    D, k, h, sig = 12, 21, 7, [6007]
    seqs, ids = [], []
    for d in range(D):
        L = int(rng.integers(300, 1500))
        seqs.append(np.frombuffer(b"ACGT", dtype=np.uint8)[rng.integers(0, 4, L)].tobytes())
        ids.append(d)
    ob = oracle_mod.CobsBank.empty(sig, (D + 7) // 8, D, h, k)
    ob.build(seqs, ids)
    gb = xs.Bank.create_cobs(k, h, sig, D, [f"sp{i}" for i in range(D)])
    gb.upload(ob.rows)
    path = tmp_path / "index.cobs_classic"
    gb.save(path)
    gb.close()

    s = mod.GpuSearch(path)
    assert (s.k, s.D, s.names) == (k, D, [f"sp{i}" for i in range(D)])
    reads = [q[o:o + 150].decode() for q in seqs for o in (0, 100)] + ["ACGT", ""]
    reuse = np.zeros((len(reads), D), np.uint32)
    for step in (1, 3):
        got, nk = s.search_batch(reads, step)
        want, want_n = ob.query([r.encode() for r in reads], step=step)
        assert np.array_equal(got, want.reshape(got.shape)) and np.array_equal(nk, want_n)
        got2, _ = s.search_batch(reads, step, out=reuse)        # a serving loop's reused matrix
        assert got2 is reuse and np.array_equal(reuse, want.reshape(got.shape))
    with pytest.raises(ValueError):
        s.search_batch(reads, 1, out=np.zeros((len(reads), D), np.uint16))
    res = s.search(reads[0])
    assert res[0].doc_name == "sp0" and res[0].score == 130
    assert [r.score for r in res] == sorted((r.score for r in res), reverse=True)
    # the reference's consumers of cobs_index.SearchResult run unchanged on it
    for q in reads[:6]:
        res = s.search(q)
        row = ob.query([q.encode()])[0][0]
        conv = _convert_cobs_result_to_dict(res)
        assert list(conv) == [f"sp{d}" for d in sorted(range(D), key=lambda d: (-int(row[d]), d))]
        assert conv == {f"sp{d}": int(row[d]) for d in range(D)}
        assert get_cobs_result(res, False) == conv
        assert get_cobs_result(res, True) == {n: v for n, v in conv.items() if v > 50}
    del s

    nbytes, K = oracle_mod.BloomFilter.params(20_000, 0.01)
    bf = oracle_mod.BloomFilter(np.zeros(nbytes, dtype=np.uint8), K, k)
    bf.build(seqs)
    gbl = xs.Bank.create_bloom(k, nbytes, K)
    gbl.upload(bf.bits)
    gbl.save(tmp_path / "filter.bloom")
    gbl.close()
    s = mod.GpuSearch(tmp_path / "filter.bloom", mod.RBLOOM, term_size=k)
    got, nk = s.search_batch(reads)
    want, want_n = bf.query([r.encode() for r in reads])
    assert np.array_equal(got[:, 0], want) and np.array_equal(nk, want_n)
