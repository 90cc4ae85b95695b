"""Config 3 and config 5 end to end over gloo on CPU (world 2, 3 and 8).

* Config 3: ``distributed.classify_species_sharded`` — every rank parses only
  its byte range of one FASTQ file, probes it, the D+1 totals are
  all-reduced, rank 0 forms the SVM label, every rank writes a JSON shard.
  The merged shards must equal the single-process result of the same model
  (``predict_columnar`` + ``save``, the reference's classify_species flow,
  src/xspect/classify.py:43-92), for plain and SVM models, exclusions,
  display names, steps, and more ranks than the file has reads.
* Config 5: a multi-genus set of 120 documents sharded over the ranks (one
  bank of 40-50 docs each): the gathered hit matrix equals the bank-by-bank
  concatenation.

The per-rank probe is the CPU oracle behind the model's index interface
(test infrastructure); on MI355X the same functions run on the HIP banks
with RCCL (tests/test_gpu_distributed.py, tools/gpu/gpu_r03_sharded.sh).
"""
from __future__ import annotations

import json
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
K = 21


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _Info:
    device = 0


class OracleIndex:
    """The Bank interface predict_columnar uses, answered by the CPU oracle."""

    def __init__(self, ob, names):
        self.ob, self.doc_names, self.num_docs, self.info = ob, list(names), len(names), _Info()

    def query(self, packed, step=1, hit_dtype=np.uint32):
        from xspect2_amd.bank import max_kmers, narrowest_count_dtype
        h, nk = self.ob.query_packed(np.ascontiguousarray(packed.buf), np.ascontiguousarray(packed.offsets),
                                     step=step, threads=1)
        if hit_dtype == "auto":  # as Bank.query: the narrowest exact type
            hit_dtype = narrowest_count_dtype(max_kmers(packed, self.ob.k, step))
        return h.astype(hit_dtype), nk


def _setup(tmp: Path, n_reads: int, svm: bool, write: bool = True, id_mod: int = 0, short_at: int = -1,
           mis_at: int = -1, name: str = "misclassified"):
    """A species model over 6 synthetic genomes (oracle bank), its reads as a
    FASTQ file (written by the parent before the ranks start: a rank must not
    rewrite a file another rank is reading)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel
    from xspect2_amd.probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    rng = np.random.default_rng(7)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    genomes = [acgt[rng.integers(0, 4, 3000)].tobytes() for _ in range(6)]
    names = [f"GCF_{470 + 13 * d:09d}" for d in range(6)]
    ob = oracle.CobsBank.empty([oracle.signature_size(3000, 7, 0.01)], 1, 6, 7, K)
    ob.build(genomes, list(range(6)))
    base = tmp / "models"
    if svm:
        model = ProbabilisticFilterSVMModel(K, "Acinetobacter", None, None, "Species", base, "rbf", 1.0)
        (base / model.slug()).mkdir(parents=True, exist_ok=True)
        rows = ["file," + ",".join(sorted(names)) + ",label_id"]
        for j, lab in enumerate(sorted(names)):
            for rep in range(3):
                v = [round(0.05 + 0.02 * rep, 2)] * 6
                v[j] = 1.0 - 0.1 * rep
                rows.append(f"acc{j}{rep}," + ",".join(str(x) for x in v) + f",{lab}")
        if write:
            (base / model.slug() / "scores.csv").write_text("\n".join(rows))
    else:
        model = ProbabilisticFilterModel(K, "Acinetobacter", None, None, "Species", base)
    model.display_names = {n: f"Acinetobacter sp{d}" for d, n in enumerate(names)}
    model.index = OracleIndex(ob, names)
    reads = []
    for i in range(n_reads):
        g = genomes[i % 6] if i % 7 else acgt[rng.integers(0, 4, 3000)].tobytes()
        L = int(rng.integers(K + 1, 200)) if i != short_at else K  # len <= k: the reference raises
        s = int(rng.integers(0, len(g) - L))
        rid = name if i == mis_at else f"read_{i % id_mod if id_mod else i}"
        reads.append((rid, g[s:s + L].decode()))
    fq = tmp / "reads.fq"
    if write:
        fq.write_text("".join(f"@{rid} x\n{s}\n+\n{'I' * len(s)}\n" for rid, s in reads))
    return model, fq


CASES = [dict(step=1), dict(step=3, display_name=True), dict(step=1, exclude_ids=["GCF_000000483"])]


def _worker(rank: int, world: int, port: int, tmp: str, n_reads: int, svm: bool):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, fq = _setup(Path(tmp), n_reads, svm, write=False)
        for i, kw in enumerate(CASES):
            distributed.classify_species_sharded(model, fq, Path(tmp) / "out" / f"case{i}.json", **kw)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_reads,svm", [(2, 600, False), (3, 600, True), (3, 2, True), (8, 1000, True)])
def test_classify_species_sharded_equals_single_process(tmp_path, world, n_reads, svm):
    import torch.multiprocessing as mp
    from xspect2_amd import distributed

    model, fq = _setup(tmp_path, n_reads, svm)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), n_reads, svm), nprocs=world, join=True)
    for i, kw in enumerate(CASES):
        res = model.predict_columnar(fq, **kw)
        res.input_source = fq.name
        res.save(tmp_path / f"single{i}.json")
        want = json.loads((tmp_path / f"single{i}.json").read_text())
        shards = [distributed.shard_path(tmp_path / "out" / f"case{i}.json", r, world) for r in range(world)]
        assert all(p.exists() for p in shards)
        got = distributed.merge_result_shards(shards)
        assert got == want
        assert list(got["hits"]) == list(want["hits"])
        distributed.merge_result_files(shards, tmp_path / f"merged{i}.json")
        assert (tmp_path / f"merged{i}.json").read_bytes() == (tmp_path / f"single{i}.json").read_bytes()
        if svm:
            assert got["prediction"] == want["prediction"]
        per_shard = [len(json.loads(p.read_text())["hits"]) for p in shards]
        assert sum(per_shard) == n_reads
        if n_reads >= 600:
            assert min(per_shard) > n_reads / world / 2  # byte ranges balance the reads


def _dup_worker(rank: int, world: int, port: int, tmp: str, n_reads: int, id_mod: int, short_at: int):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, fq = _setup(Path(tmp), n_reads, True, write=False, id_mod=id_mod, short_at=short_at)
        try:
            distributed.classify_species_sharded(model, fq, Path(tmp) / "out" / "dup.json")
            (Path(tmp) / f"rank{rank}.txt").write_text("ok")
        except Exception as e:  # noqa: BLE001
            (Path(tmp) / f"rank{rank}.txt").write_text(f"{type(e).__name__}: {e}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,id_mod", [(3, 350), (2, 7), (3, 1)])
def test_repeated_ids_across_shards_follow_the_reference_dict(tmp_path, world, id_mod):
    """Read ids that repeat in different shards (ids read_{i % id_mod}: 600
    reads, so each id occurs in 2 to 600 records spread over the ranks): the
    merged shards equal the single-process JSON, whose dictionaries keep one
    entry per id at its first record with its last record's values
    (probabilistic_filter_model.py:310) and sum the totals over them
    (result.py:76-90); the SVM label follows those totals."""
    import torch.multiprocessing as mp
    from xspect2_amd import distributed

    n_reads = 600
    model, fq = _setup(tmp_path, n_reads, True, id_mod=id_mod)
    mp.spawn(_dup_worker, args=(world, _free_port(), str(tmp_path), n_reads, id_mod, -1), nprocs=world, join=True)
    assert all((tmp_path / f"rank{r}.txt").read_text() == "ok" for r in range(world))
    res = model.predict_columnar(fq)
    res.input_source = fq.name
    res.save(tmp_path / "single.json")
    want = json.loads((tmp_path / "single.json").read_text())
    shards = [distributed.shard_path(tmp_path / "out" / "dup.json", r, world) for r in range(world)]
    got = distributed.merge_result_shards(shards)
    assert len(want["hits"]) == min(id_mod, n_reads)
    assert got == want
    assert list(got["hits"]) == list(want["hits"])
    assert got["prediction"] == want["prediction"]
    assert sum(len(json.loads(p.read_text())["hits"]) for p in shards) == len(want["hits"])
    distributed.merge_result_files(shards, tmp_path / "merged.json")
    assert (tmp_path / "merged.json").read_bytes() == (tmp_path / "single.json").read_bytes()


def _mis_worker(rank: int, world: int, port: int, tmp: str, n_reads: int, mis_at: int, name: str = "misclassified"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, fq = _setup(Path(tmp), n_reads, True, write=False, mis_at=mis_at, name=name)
        try:
            distributed.classify_species_sharded(model, fq, Path(tmp) / "out" / "mis.json")
            (Path(tmp) / f"rank{rank}.txt").write_text("ok")
        except Exception as e:  # noqa: BLE001
            (Path(tmp) / f"rank{rank}.txt").write_text(f"{type(e).__name__}: {e}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mis_at", [(3, 595), (2, 0), (3, 300)])
def test_read_named_misclassified_in_any_shard(tmp_path, world, mis_at):
    """A read literally named "misclassified" is popped from the reference's
    hits into the result's "misclassified" field (result.py:43): it leaves the
    per-doc totals and the choice of the first row that orders "total", but
    keeps its k-mers in num_kmers.  Whichever shard holds it (the last, the
    first as its first read, a middle one), the merged shards equal the
    single-process JSON."""
    import torch.multiprocessing as mp
    from xspect2_amd import distributed

    n_reads = 600
    model, fq = _setup(tmp_path, n_reads, True, mis_at=mis_at)
    mp.spawn(_mis_worker, args=(world, _free_port(), str(tmp_path), n_reads, mis_at), nprocs=world, join=True)
    res = model.predict_columnar(fq)
    res.input_source = fq.name
    res.save(tmp_path / "single.json")
    want = json.loads((tmp_path / "single.json").read_text())
    assert want["misclassified"] is not None and "misclassified" not in want["hits"]
    shards = [distributed.shard_path(tmp_path / "out" / "mis.json", r, world) for r in range(world)]
    assert distributed.merge_result_shards(shards) == want
    distributed.merge_result_files(shards, tmp_path / "merged.json")
    assert (tmp_path / "merged.json").read_bytes() == (tmp_path / "single.json").read_bytes()


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world,at", [(3, 590), (2, 0)])
def test_read_named_total_raises_on_every_rank(tmp_path, world, at):
    """A read named "total" is the reference's reserved key (result.py:33-36:
    ValueError); in whichever shard it falls, every rank raises that error
    instead of the others waiting in the totals' all-reduce."""
    import torch.multiprocessing as mp
    from xspect2_amd.result import ModelResult
    n_reads = 600
    with pytest.raises(ValueError) as want:
        ModelResult("m", {"total": {"a": 1}}, {"total": 1})
    _setup(tmp_path, n_reads, True, mis_at=at, name="total")
    mp.spawn(_mis_worker, args=(world, _free_port(), str(tmp_path), n_reads, at, "total"), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == f"ValueError: {want.value}"


def _empty_worker(rank: int, world: int, port: int, tmp: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch.distributed as dist
    from xspect2_amd import distributed

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        model, _ = _setup(Path(tmp), 10, True, write=False)
        try:
            distributed.classify_species_sharded(model, Path(tmp) / "empty.fq", Path(tmp) / "out" / "e.json")
            (Path(tmp) / f"rank{rank}.txt").write_text("ok")
        except Exception as e:  # noqa: BLE001
            (Path(tmp) / f"rank{rank}.txt").write_text(f"{type(e).__name__}: {e}")
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(180)
def test_empty_input_raises_index_error_on_every_rank(tmp_path):
    """An input without records: the reference's get_total_hits indexes the
    first hit row of an empty dict (result.py:86, IndexError); the sharded job
    raises that on every rank, as one process's save does."""
    import torch.multiprocessing as mp
    model, _ = _setup(tmp_path, 10, True)
    (tmp_path / "empty.fq").write_text("")
    with pytest.raises(IndexError) as want:  # the SVM model's predict already asks for the totals
        model.predict_columnar(tmp_path / "empty.fq").save(tmp_path / "single.json")
    mp.spawn(_empty_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        assert (tmp_path / f"rank{r}.txt").read_text() == f"IndexError: {want.value}"


@pytest.mark.timeout(180)
@pytest.mark.parametrize("world", [2, 3])
def test_an_error_on_one_rank_raises_on_every_rank(tmp_path, world):
    """Only the last shard holds a read no longer than k: every rank raises the
    reference's ValueError instead of the others waiting in the totals'
    all-reduce."""
    import torch.multiprocessing as mp

    n_reads = 300
    _setup(tmp_path, n_reads, True, short_at=n_reads - 2)
    mp.spawn(_dup_worker, args=(world, _free_port(), str(tmp_path), n_reads, 0, n_reads - 2), nprocs=world,
             join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ValueError: Invalid sequence, must be longer than k"


def _gather_worker(rank: int, world: int, port: int, tmp: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    import torch
    import torch.distributed as dist
    from xspect2_amd import distributed
    from xspect2_amd.packing import pack_sequences

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        banks, reads = _genera(oracle, world)
        pr = pack_sequences(reads)
        ob = banks[rank]
        hits, nk = distributed.docs_sharded_hits(
            pr, 1, lambda sl, st: ob.query_packed(sl.buf, sl.offsets, step=st, threads=1))
        # the tensor-level gather the device path uses, from a CPU tensor
        h, _ = ob.query_packed(pr.buf, pr.offsets, step=2, threads=1)
        t = distributed.gather_doc_shards(torch.from_numpy(h.view(np.int32)), 130)
        np.savez(Path(tmp) / f"g{rank}.npz", hits=hits, nk=nk, step2=t.numpy().view(np.uint32))
    finally:
        dist.destroy_process_group()


def _genera(oracle, world):
    """`world` genus banks of 40-50 species (> 100 docs in all), reads from all of them."""
    rng = np.random.default_rng(5)
    acgt = np.frombuffer(b"ACGT", dtype=np.uint8)
    banks, reads = [], []
    for g in range(world):
        D = 40 + 5 * g
        docs = [acgt[rng.integers(0, 4, 800)].tobytes() for _ in range(D)]
        ob = oracle.CobsBank.empty([oracle.signature_size(800, 7, 0.01)], (D + 7) // 8, D, 7, K)
        ob.build(docs, list(range(D)))
        banks.append(ob)
        reads += [d[o:o + 150] for d in docs[::3] for o in (0, 500)]
    reads += [acgt[rng.integers(0, 4, 150)].tobytes() for _ in range(30)]
    return banks, reads


@pytest.mark.parametrize("world", [3, 8])
def test_multigenus_docs_sharded_over_100_docs(tmp_path, world):
    import torch.multiprocessing as mp
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle

    mp.spawn(_gather_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    banks, reads = _genera(oracle, world)
    assert sum(b.D for b in banks) > 100
    want1 = np.concatenate([b.query(reads)[0] for b in banks], axis=1)
    want2 = np.concatenate([b.query(reads, step=2)[0] for b in banks], axis=1)
    assert int(want1.sum()) > 0
    for r in range(world):
        o = np.load(tmp_path / f"g{r}.npz")
        assert np.array_equal(o["hits"], want1)
        assert np.array_equal(o["step2"], want2)


def _docs_worker(rank: int, world: int, port: int, tmp: str, dup: bool = False, catch: bool = False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    import torch.distributed as dist
    from xspect2_amd import distributed
    from xspect2_amd.probabilistic_filter_model import ProbabilisticFilterModel

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        banks, reads = _genera(oracle, world)
        m = ProbabilisticFilterModel(K, f"Genus{rank}", None, None, "Species", Path(tmp) / "m")
        names = [f"g{rank}_sp{d}" for d in range(banks[rank].D)]
        m.index = OracleIndex(banks[rank], names)
        try:
            distributed.classify_docs_sharded(m, Path(tmp) / "reads.fasta", Path(tmp) / "out" / "docs.json")
            (Path(tmp) / f"rank{rank}.txt").write_text("ok")
        except Exception as e:  # noqa: BLE001
            if not catch:
                raise
            (Path(tmp) / f"rank{rank}.txt").write_text(f"{type(e).__name__}: {e}")
    finally:
        dist.destroy_process_group()


def _write_reads(path: Path, reads, dup: bool):
    """FASTA of the reads; with dup, ids repeat far apart (reads i and
    i + n/2 share an id, so the repeats fall into different shards)."""
    half = (len(reads) + 1) // 2
    with open(path, "wb") as fh:
        for i, r in enumerate(reads):
            fh.write(b">r%d\n%s\n" % (i % half if dup else i, r))


@pytest.mark.parametrize("world,dup", [(2, False), (3, False), (3, True), (8, False)])
def test_predict_docs_sharded_multigenus(tmp_path, world, dup):
    """Config 5 as a library call: `world` genus models of 40-75 species
    (> 100 docs) on `world` ranks, one FASTA of reads from all of them.  Each
    rank parses its byte range, the reads are all-gathered, every rank probes
    them against its bank and the hit columns go back by all-to-all to the
    rank that owns the reads; every rank writes its own shard.  The merged
    shards equal the JSON of one process probing every bank and concatenating
    the columns, repeated ids (dup) included."""
    import torch.multiprocessing as mp
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    from xspect2_amd import distributed
    from xspect2_amd.result import MatrixResult

    banks, reads = _genera(oracle, world)
    _write_reads(tmp_path / "reads.fasta", reads, dup)
    mp.spawn(_docs_worker, args=(world, _free_port(), str(tmp_path), dup), nprocs=world, join=True)
    hits = np.concatenate([b.query(reads)[0] for b in banks], axis=1)
    nk = banks[0].query(reads)[1]
    labels = [f"g{g}_sp{d}" for g in range(world) for d in range(banks[g].D)]
    half = (len(reads) + 1) // 2
    ids = [f"r{i % half if dup else i}" for i in range(len(reads))]
    want = MatrixResult("multi-genus-docs-sharded", ids, labels, hits, nk)
    want.input_source = "reads.fasta"
    want.save(tmp_path / "want.json")
    assert len(labels) > 100 or world < 3
    shards = [distributed.shard_path(tmp_path / "out" / "docs.json", r, world) for r in range(world)]
    per_shard = [json.loads(p.read_text()) for p in shards]
    got = distributed.merge_result_shards(shards)
    w = json.loads((tmp_path / "want.json").read_text())
    assert got == w
    assert list(got["hits"]) == list(w["hits"])
    assert sum(len(d["hits"]) for d in per_shard) == len(w["hits"])  # each read in exactly one shard
    distributed.merge_result_files(shards, tmp_path / "merged.json")
    assert (tmp_path / "merged.json").read_bytes() == (tmp_path / "want.json").read_bytes()
    if not dup:
        assert min(len(d["hits"]) for d in per_shard) > 0


@pytest.mark.timeout(180)
def test_docs_sharded_error_on_one_rank_raises_on_every_rank(tmp_path):
    """Config 5: only the last rank's byte range holds a read no longer than
    k; every rank raises the reference's ValueError (a rank that
    raised alone left the others in the batch collectives)."""
    import torch.multiprocessing as mp
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle

    world = 3
    banks, reads = _genera(oracle, world)
    reads = reads + [reads[-1][:K]]  # the last record: len == k
    with open(tmp_path / "reads.fasta", "wb") as fh:
        for i, r in enumerate(reads):
            fh.write(b">r%d\n%s\n" % (i, r))
    mp.spawn(_docs_worker, args=(world, _free_port(), str(tmp_path), False, True), nprocs=world, join=True)
    for r in range(world):
        assert (tmp_path / f"rank{r}.txt").read_text() == "ValueError: Invalid sequence, must be longer than k"


def _exchange_worker(rank: int, world: int, port: int, tmp: str):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    from xspect2_amd import distributed

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(11)
        dims = [3 + 2 * r for r in range(world)]                 # D_r differ: rows padded to the widest
        counts = [int(c) for c in rng.integers(0, 40, world)]    # reads per rank (some may be 0)
        n = sum(counts)
        out = {}
        for wire, top in ((torch.uint8, 255), (torch.int16, 32767), (torch.int32, 1 << 30)):
            # every rank's full columns, from one seed: rank r holds columns of block r
            full = np.random.default_rng(5).integers(0, top + 1, (n, sum(dims)))
            c0 = sum(dims[:rank])
            mine = torch.from_numpy(full[:, c0:c0 + dims[rank]].astype(np.int32))
            got = distributed.exchange_doc_columns(mine, counts, dims, wire)
            lo = sum(counts[:rank])
            out[str(wire)] = (got.to(torch.int64).numpy(), full[lo:lo + counts[rank]])
        np.savez(Path(tmp) / f"x{rank}.npz", **{k + "_got": v[0] for k, v in out.items()},
                 **{k + "_want": v[1] for k, v in out.items()})
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_exchange_doc_columns_all_widths(tmp_path, world):
    """exchange_doc_columns over gloo: rank q ends with its reads' rows of
    every rank's columns, in 1, 2 (float16 bit patterns on the wire) and 4
    bytes, with ranks of different doc counts and of no reads."""
    import torch.multiprocessing as mp
    mp.spawn(_exchange_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        z = np.load(tmp_path / f"x{r}.npz")
        for k in ("torch.uint8", "torch.int16", "torch.int32"):
            assert np.array_equal(z[k + "_got"], z[k + "_want"]), (r, k)
