"""Multi-process collectives of xspect2_amd.distributed with gloo on CPU.

The per-rank compute is the CPU oracle here (test infrastructure); on MI355X
the same functions run with the HIP banks and RCCL (bench.py, config 3).
"""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _banks(seed: int = 0):
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    rng = np.random.default_rng(seed)
    docs = ["".join(rng.choice(list("ACGT"), 600)) for _ in range(10)]
    full = oracle.CobsBank.empty([4001], 2, 10, 3, 21)
    full.build(docs, list(range(10)))
    part_a = oracle.CobsBank.empty([2003], 1, 4, 3, 21)
    part_a.build(docs[:4], list(range(4)))
    part_b = oracle.CobsBank.empty([3001], 1, 6, 3, 21)
    part_b.build(docs[4:], list(range(6)))
    reads = [d[i:i + 150] for d in docs for i in (0, 200, 400)] + \
            ["".join(rng.choice(list("ACGTN"), 150)) for _ in range(13)]
    return oracle, full, part_a, part_b, reads


def _worker(rank: int, world: int, port: int, out_dir: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed
    from xspect2_amd.packing import pack_sequences

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        oracle, full, part_a, part_b, reads = _banks()
        pr = pack_sequences(reads)

        def local_totals(sl, step):
            h, nk = full.query_packed(sl.buf, sl.offsets, step=step, threads=1)
            return h.sum(axis=0, dtype=np.uint64), int(nk.sum())

        tot, nk = distributed.reads_sharded_totals(pr, 2, local_totals)
        lo, hi, hits, nkr, g_tot, g_nk = distributed.reads_sharded_hits(
            pr, 1, lambda sl, st: full.query_packed(sl.buf, sl.offsets, step=st, threads=1))
        mine = part_a if rank % 2 == 0 else part_b
        dh, _ = distributed.docs_sharded_hits(
            pr, 1, lambda sl, st: mine.query_packed(sl.buf, sl.offsets, step=st, threads=1))
        # reads long enough for 2-byte (6,000 bp) and 4-byte (36,000 bp) transport
        long_reads = reads[:3] + ["".join(reads[i] for i in range(30)) * 2, "".join(reads[:30]) * 12]
        dl = [distributed.docs_sharded_hits(
                  pack_sequences(rs), 1, lambda sl, st: mine.query_packed(sl.buf, sl.offsets, step=st, threads=1))[0]
              for rs in (long_reads[:4], long_reads)]  # int16, then int32 transport
        labels = [f"sp{d:02d}" for d in range(10)][::-1]  # label order differs from doc order
        pred = distributed.reads_sharded_svm_predict(
            pr, 1, labels, lambda sl, st: local_totals(sl, st),
            lambda x: "|".join(f"{v:.2f}" for v in x[0]))  # the vector itself, as the "label"
        np.savez(Path(out_dir) / f"r{rank}.npz", tot=tot, nk=nk, lo=lo, hi=hi, hits=hits,
                 g_tot=g_tot, g_nk=g_nk, dh=dh, dl16=dl[0], dl32=dl[1],
                 pred=np.array(pred))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_reads_and_docs_sharded(tmp_path, world):
    import torch.multiprocessing as mp

    port = _free_port()
    mp.spawn(_worker, args=(world, port, str(tmp_path)), nprocs=world, join=True)
    oracle, full, part_a, part_b, reads = _banks()
    want_h1, want_n1 = full.query(reads, step=1)
    want_h2, want_n2 = full.query(reads, step=2)
    outs = [np.load(tmp_path / f"r{r}.npz") for r in range(world)]
    for o in outs:
        # reads sharded, bank replicated: all-reduced totals equal the single-process totals
        assert np.array_equal(o["tot"], want_h2.sum(axis=0, dtype=np.uint64))
        assert int(o["nk"]) == int(want_n2.sum())
        assert np.array_equal(o["g_tot"], want_h1.sum(axis=0, dtype=np.uint64))
        assert int(o["g_nk"]) == int(want_n1.sum())
    # per-read rows of each shard are the rows of the whole query
    stitched = np.concatenate([o["hits"] for o in outs], axis=0)
    assert np.array_equal(stitched, want_h1)
    # docs sharded: rank r holds part_a (even r) or part_b (odd r); columns in rank order
    ha, _ = part_a.query(reads)
    hb, _ = part_b.query(reads)
    want = np.concatenate([ha if r % 2 == 0 else hb for r in range(world)], axis=1)
    for o in outs:
        assert np.array_equal(o["dh"], want)
    long_reads = reads[:3] + ["".join(reads[i] for i in range(30)) * 2, "".join(reads[:30]) * 12]
    for key, rs in (("dl16", long_reads[:4]), ("dl32", long_reads)):
        ha, na = part_a.query(rs)
        hb, _ = part_b.query(rs)
        assert 255 < int(na.max()) <= 32767 if key == "dl16" else int(na.max()) > 32767
        assert int(ha.max()) > 255  # counts that do not fit a byte travel intact
        want_l = np.concatenate([ha if r % 2 == 0 else hb for r in range(world)], axis=1)
        for o in outs:
            assert np.array_equal(o[key], want_l)
    # SVM vector from the all-reduced totals, formed on rank 0 and broadcast,
    # equals the single-process ModelResult total scores in label order
    from xspect2_amd.result import ModelResult
    labels = [f"sp{d:02d}" for d in range(10)][::-1]
    hits = {f"r{i}": {labels[d]: int(want_h1[i, d]) for d in range(10)} for i in range(len(reads))}
    res = ModelResult("m", hits, {f"r{i}": int(n) for i, n in enumerate(want_n1)})
    vec = [v for _, v in sorted(res.get_scores()["total"].items())]
    for o in outs:
        assert str(o["pred"]) == "|".join(f"{v:.2f}" for v in vec)
