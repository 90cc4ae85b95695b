"""One COBS classic bank column-split over ranks (SURVEY.md §8(e) config 5,
option b; xs_bank_open_docs): each slice holds the byte columns of docs
[lo, hi) of every row, so the slices' hit matrices side by side are the whole
bank's, bit for bit, and equal the oracle's (GPU).  The multi-rank call
(distributed.predict_bank_sharded over load_docs_slice) is checked at world 1
under RCCL here and at N = 2 by tools/sharded_classify.py bank-* on the box."""
from __future__ import annotations

import socket

import numpy as np
import pytest

from test_gpu_parity import _pair, _reads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def xs():
    from xspect2_amd import _lib
    from xspect2_amd import bank as bank_mod
    assert _lib.device_count() >= 1
    return bank_mod


@pytest.mark.parametrize("D,k,h,sig", [(100, 21, 7, [40_000]), (300, 16, 3, [7_919]), (2100, 21, 7, [4_001]),
                                       (13, 31, 1, [2_003])])
def test_slices_side_by_side_are_the_whole_bank(xs, oracle_mod, tmp_path, D, k, h, sig):
    from xspect2_amd import _lib
    from xspect2_amd.distributed import cobs_classic_docs, doc_slice
    ob, gb, seqs, _ = _pair(xs, oracle_mod, D, k, h, sig, seed=D)
    path = tmp_path / "index.cobs_classic"
    gb.save(path)
    assert cobs_classic_docs(path) == D
    rng = np.random.default_rng(D + 1)
    reads = _reads(rng, 200, k) + [s[:300] for s in seqs[:20]] + [b"", b"A" * (k - 1), seqs[0] * 2]
    want_h, want_n = ob.query(reads, step=2)
    R = (D + 7) // 8
    for world in sorted({1, 2, 3, min(8, R)}):
        if world > R:
            continue
        parts = []
        for r in range(world):
            lo, hi = doc_slice(D, r, world)
            b = xs.Bank.open(path, _lib.XS_BANK_COBS_CLASSIC, docs=(lo, hi))
            assert b.num_docs == hi - lo and b.doc_names == gb.doc_names[lo:hi]
            hh, nn = b.query(reads, step=2)
            assert np.array_equal(nn, want_n)
            parts.append(hh)
            b.close()
        assert np.array_equal(np.concatenate(parts, axis=1), want_h), world
    for bad in ((4, D), (0, D + 8), (8, 8), (0, 4) if D > 8 else (1, D)):
        with pytest.raises(_lib.XsError):
            xs.Bank.open(path, _lib.XS_BANK_COBS_CLASSIC, docs=bad)
    with pytest.raises(ValueError):
        xs.Bank.open(path, _lib.XS_BANK_COBS_COMPACT, docs=(0, 8))
    gb.close()


def test_predict_bank_sharded_world1(tmp_path, monkeypatch):
    """load_docs_slice + predict_bank_sharded under RCCL at world 1 (the whole
    bank as the one slice): the model's own columnar prediction, its slug."""
    import torch
    import torch.distributed as dist
    from xspect2_amd import distributed
    from xspect2_amd.file_io import Record, write_fasta
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    from xspect2_amd.synth import make_genomes

    genomes = [g.tobytes().decode() for g in make_genomes(20, 20_000, seed=7)]
    sdir = tmp_path / "sp"
    sdir.mkdir()
    for i, g in enumerate(genomes):
        write_fasta([Record(f"c{i}", g)], sdir / f"{100 + i}.fasta")
    m = ProbabilisticFilterModel(21, "Genus", None, None, "Species", tmp_path / "models")
    m.fit(sdir)
    m.save()
    fq = tmp_path / "r.fq"
    fq.write_text("".join(f"@r{j}\n{g[o:o + 150]}\n+\n{'I' * 150}\n" for j, g in enumerate(genomes)
                          for o in (0, 7000, 15000)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        sl = distributed.load_docs_slice(ProbabilisticFilterModel, tmp_path / "models" / "genus-species.json")
        res = distributed.predict_bank_sharded(sl, fq)
        want = m.predict_columnar(fq)
        want.input_source = fq.name
        res.save(tmp_path / "a.json")
        want.save(tmp_path / "b.json")
        assert (tmp_path / "a.json").read_bytes() == (tmp_path / "b.json").read_bytes()
        sl.close()
    finally:
        dist.destroy_process_group()
    m.close()
