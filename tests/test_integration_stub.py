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
    for step in (1, 3):
        got, nk = s.search_batch(reads, step)
        want, want_n = ob.query([r.encode() for r in reads], step=step)
        assert np.array_equal(got, want.reshape(got.shape)) and np.array_equal(nk, want_n)
    res = s.search(reads[0])
    assert [n for _, n in res][0] == "sp0" and res[0][0] == 130
    assert [sc for sc, _ in res] == sorted((sc for sc, _ in res), reverse=True)
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
