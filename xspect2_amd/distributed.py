"""Multi-GPU probe: one process per GPU, torch.distributed (RCCL on ROCm).

Two partitionings:

* **reads sharded, bank replicated** (config 3) — each rank classifies a
  contiguous share of the reads against its own replica of the bank; the
  only exchange is one all-reduce (sum) of D+1 counters (per-doc totals and
  the k-mer total), the inputs of ``ModelResult.get_scores()["total"]`` and
  the SVM vector.  Per-read hit rows stay on the rank that computed them.
  ``classify_species_sharded`` is the whole flow for one input file: every
  rank parses only its byte range of the file (xs_fastx_open_range), the
  totals are all-reduced on a device tensor, rank 0 forms the SVM vector and
  label, and every rank writes its own JSON shard.
* **docs sharded** (config 5) — each rank holds a different bank (e.g. one
  genus of a multi-genus collection) and probes all reads; per-read hit
  vectors are all-gathered along the doc axis, in the narrowest integer type
  that carries them (``docs_sharded_hits_device`` stays on the device from
  the probe to the gathered matrix).

The collectives run on CUDA tensors when the process group is RCCL
(``nccl``) and on CPU tensors under ``gloo`` (CPU tests, and the one-GPU
rehearsal where several ranks share a device).  The per-rank compute of the
host-level helpers is a callable so they can be exercised with the CPU oracle.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Callable

import numpy as np

from .packing import PackedIds, PackedReads


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of n items for `rank` (sizes differ by <= 1)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def slice_reads(reads: PackedReads, lo: int, hi: int) -> PackedReads:
    offs = reads.offsets[lo:hi + 1]
    a, b = int(offs[0]), int(offs[-1])
    buf = np.concatenate([reads.buf[a:b], np.zeros(1, dtype=np.uint8)])
    return PackedReads(buf, (offs - offs[0]).astype(np.uint64))


def _dist():
    import torch.distributed as dist
    return dist


def collective_device():
    """Where collective tensors live: the current GPU under RCCL, else the CPU."""
    import torch
    dist = _dist()
    if dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _on_wire(t):
    """`t` moved to the collective device (a no-op when it is already there)."""
    dev = collective_device()
    return t if t.device == dev else t.to(dev)


def allreduce_(t, op=None):
    """In-place all-reduce of a tensor on any device (RCCL on the device, or
    gloo through a host copy)."""
    dist = _dist()
    op = dist.ReduceOp.SUM if op is None else op
    w = _on_wire(t)
    dist.all_reduce(w, op=op)
    if w is not t:
        t.copy_(w)
    return t


def allreduce_totals(totals: np.ndarray, total_kmers: int, device=None) -> tuple[np.ndarray, int]:
    """Sum of (per-doc totals, k-mer total) over all ranks (one collective)."""
    import torch
    t = torch.from_numpy(np.concatenate([totals.astype(np.int64), [np.int64(total_kmers)]]))
    if device is not None:
        t = t.to(device)
    allreduce_(t)
    out = t.cpu().numpy().view(np.uint64)
    return out[:-1].copy(), int(out[-1])


def reads_sharded_totals(reads: PackedReads, step: int,
                         local_totals: Callable[[PackedReads, int], tuple[np.ndarray, int]],
                         device=None) -> tuple[np.ndarray, int]:
    """Config 3: every rank probes its slice; totals are all-reduced."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(reads.n, rank, world)
    tot, nk = local_totals(slice_reads(reads, lo, hi), step)
    return allreduce_totals(np.asarray(tot, dtype=np.uint64), nk, device)


def reads_sharded_hits(reads: PackedReads, step: int,
                       local_query: Callable[[PackedReads, int], tuple[np.ndarray, np.ndarray]],
                       device=None):
    """Config 3 with per-read rows: (lo, hi, local hits, local num_kmers, global totals, N)."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    lo, hi = shard_range(reads.n, rank, world)
    hits, nk = local_query(slice_reads(reads, lo, hi), step)
    tot = hits.sum(axis=0, dtype=np.uint64) if hits.size else np.zeros(hits.shape[1], np.uint64)
    g_tot, g_nk = allreduce_totals(tot, int(np.asarray(nk, dtype=np.uint64).sum()), device)
    return lo, hi, hits, nk, g_tot, g_nk


def transport_dtype(max_count: int):
    """Narrowest torch dtype that carries hit counts up to `max_count` exactly.

    A read's count for a doc is at most its number of sampled k-mers, so
    150 bp reads (130 k-mers) travel as one byte per (read, doc) instead of
    four: the docs-sharded all-gather moves a quarter of the bytes over xGMI."""
    import torch
    if max_count <= 255:
        return torch.uint8
    if max_count <= 32767:
        return torch.int16
    return torch.int32


def doc_shard_layout(d_local: int, max_count: int):
    """(docs of every rank, transport dtype) of a docs-sharded gather: one
    small all-gather of (D_r, largest per-read k-mer count).  It depends only
    on the banks and the reads' length class, so a serving loop computes it
    once and passes it to every ``gather_doc_shards``."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    meta = torch.tensor([int(d_local), int(max_count)], dtype=torch.int64)
    allmeta = [torch.zeros(2, dtype=torch.int64, device=collective_device()) for _ in range(world)]
    dist.all_gather(allmeta, _on_wire(meta))
    dims = [int(m[0].item()) for m in allmeta]
    return dims, transport_dtype(max(int(m[1].item()) for m in allmeta))


def gather_doc_shards(hits, max_count: int | None = None, layout=None):
    """All-gather per-rank hit columns [n, D_r] (any integer tensor, any
    device) into [n, sum(D_r)] int32 in rank order, on the tensor's device.

    The rows travel in ``transport_dtype`` of the largest per-read k-mer count
    on any rank, padded to the widest D_r (``layout`` from
    ``doc_shard_layout``, agreed by one small all-gather when not given); the
    narrowing and widening run where the tensor is (on the GPU for the
    device-resident path)."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    n, d_local = hits.shape
    dims, dt = layout if layout is not None else doc_shard_layout(d_local, max_count)
    if dims[dist.get_rank()] != d_local:
        raise ValueError("layout does not match this rank's hit columns")
    d_max = max(dims)
    pad = torch.zeros((n, d_max), dtype=dt, device=hits.device) if d_local < d_max else None
    if pad is None:
        pad = hits.to(dt)  # lossless: counts <= k-mers per read <= max_count
    else:
        pad[:, :d_local] = hits.to(dt)
    # gloo and RCCL gather no int16: 2-byte rows travel as float16 bit patterns
    # (an all-gather copies bits, it does no arithmetic)
    wire = _on_wire(pad.view(torch.float16) if dt == torch.int16 else pad)
    parts = [torch.empty_like(wire) for _ in range(world)]
    dist.all_gather(parts, wire)
    # widened straight into the output: one pass over the gathered bytes
    out = torch.empty((n, sum(dims)), dtype=torch.int32, device=hits.device)
    c0 = 0
    for p, d in zip(parts, dims):
        if dt == torch.int16:
            p = p.view(torch.int16)
        out[:, c0:c0 + d].copy_(p[:, :d])
        c0 += d
    return out


def docs_sharded_hits(reads: PackedReads, step: int,
                      local_query: Callable[[PackedReads, int], tuple[np.ndarray, np.ndarray]],
                      device=None) -> tuple[np.ndarray, np.ndarray]:
    """Config 5 from host reads: each rank's bank covers its own docs; the
    hit columns of all ranks [n, sum(D_r)] in rank order (host uint32)."""
    import torch
    hits, nk = local_query(reads, step)
    nk = np.asarray(nk)
    t = torch.from_numpy(np.ascontiguousarray(hits).view(np.int32))
    if device is not None:
        t = t.to(device)
    out = gather_doc_shards(t, int(nk.max()) if nk.size else 0)
    return out.cpu().numpy().view(np.uint32), nk


def docs_sharded_hits_device(bank, d_seqs, seq_bytes: int, d_offsets, n: int, step: int = 1, stream=None):
    """Config 5 on the device: probe device-resident reads against this rank's
    bank (xs_query_device), then all-gather the hit columns of every rank over
    RCCL, narrowed to the smallest exact type on the device and widened back
    there.  Returns (hits [n, sum(D_r)] int32, num_kmers [n] int64), both on
    the bank's device; nothing crosses to the host but two 16-byte metadata
    exchanges."""
    import torch
    dev = torch.device("cuda", bank.info.device)
    d_hits = torch.empty((n, bank.num_docs), dtype=torch.int32, device=dev)
    d_nk = torch.empty(n, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream(dev) if stream is None else stream
    bank.query_device(d_seqs, seq_bytes, d_offsets, n, step, d_hits, d_nk, None, stream=s.cuda_stream)
    with torch.cuda.stream(s):
        mx = d_nk.max().reshape(1) if n else torch.zeros(1, dtype=torch.int64, device=dev)
        allreduce_(mx, _dist().ReduceOp.MAX)
        return gather_doc_shards(d_hits, int(mx.item())), d_nk


def svm_vector(labels: list[str], totals, total_kmers: int) -> list[float]:
    """The SVM feature row from whole-job totals: round(T_d / N, 2) in label
    order (probabilistic_filter_svm_model.py:212-213 over result.py:57-72)."""
    scores = {lab: round(int(t) / total_kmers, 2) for lab, t in zip(labels, totals)}
    return [scores[lab] for lab in sorted(scores)]


def reads_sharded_svm_predict(reads: PackedReads, step: int, labels: list[str],
                              local_totals: Callable[[PackedReads, int], tuple[np.ndarray, int]],
                              classify: Callable[[list[list[float]]], object], device=None) -> str:
    """Config 3 end to end: every rank probes its slice, the D+1 totals are
    all-reduced, rank 0 forms the SVM vector and classifies it, and the label
    is broadcast to every rank."""
    tot, nk = reads_sharded_totals(reads, step, local_totals, device)
    dist = _dist()
    out = [None]
    if dist.get_rank() == 0:
        out[0] = str(classify([svm_vector(labels, tot, nk)]))
    dist.broadcast_object_list(out, src=0)
    return out[0]


# ---------------------------------------------------------------- config 3: sharded classify
def shard_path(output_path: Path, rank: int, world: int) -> Path:
    """JSON shard of one rank: <stem>.part<rank+1>-of-<world><suffix>."""
    output_path = Path(output_path)
    return output_path.with_name(f"{output_path.stem}.part{rank + 1}-of-{world}{output_path.suffix}")


def _job_first_row(res, D: int) -> np.ndarray:
    """Hit row of the job's first read (first read of the lowest rank that has
    one), which orders the labels of the job's "total" scores as the
    reference's get_total_hits does (result.py:84-90)."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    flags = [torch.zeros(1, dtype=torch.int64, device=collective_device()) for _ in range(world)]
    dist.all_gather(flags, _on_wire(torch.tensor([len(res.ids)], dtype=torch.int64)))
    owners = [r for r, f in enumerate(flags) if int(f.item()) > 0]
    if not owners:
        raise IndexError("list index out of range")  # get_total_hits on no reads, as the reference
    row = torch.zeros(D, dtype=torch.int64)
    if dist.get_rank() == owners[0]:
        row = torch.from_numpy(res.hits[0].astype(np.int64))
    row = _on_wire(row)
    dist.broadcast(row, src=owners[0])
    return row.cpu().numpy().astype(np.uint32)


def classify_species_sharded(model, input_file: Path, output_path: Path, step: int = 1,
                             display_name: bool = False, exclude_ids: list[str] | None = None):
    """Config 3 (reads sharded over the ranks of the process group), for one
    FASTA/FASTQ file and a loaded species model (the reference's
    ``classify_species``, src/xspect/classify.py:43-92, and
    ``ProbabilisticFilterSVMModel.predict``, probabilistic_filter_svm_model.py:
    175-223, spread over ranks):

    1. rank r parses only part r of the file (record-aligned byte ranges) and
       probes it against its bank replica (``predict_columnar``);
    2. the D+1 counters (per-doc totals, k-mer total) are all-reduced as one
       int64 tensor on the device (RCCL);
    3. rank 0 forms the SVM vector from the job's total scores and predicts
       the label (SVM models), which is broadcast;
    4. every rank writes its JSON shard (``shard_path``): its own reads' hits,
       scores and k-mer counts, the job's "total" and prediction.

    ``merge_result_shards`` of the shards equals the single-process JSON.
    One deviation: a read id repeated in two different shards is kept once
    per shard in the job's totals, where the single-process dictionaries keep
    only its last record (repeats inside one shard collapse as there).
    Returns this rank's MatrixResult (a shard)."""
    import torch
    from .file_io import FileShard
    from .probabilistic_filter_model import ProbabilisticFilterModel

    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    input_file = Path(input_file)
    res = ProbabilisticFilterModel.predict_columnar(model, FileShard(input_file, rank, world), exclude_ids, step,
                                                    display_name)
    D = len(res.labels)
    local = np.zeros(D + 1, dtype=np.int64)
    if res.ids:
        local[:D] = res.hits.sum(axis=0, dtype=np.uint64).astype(np.int64)
        local[D] = int(res.num_kmers.sum())
    dev = torch.device("cuda", model.index.info.device) if collective_device().type == "cuda" else None
    t = torch.from_numpy(local)
    if dev is not None:
        t = t.to(dev)
    allreduce_(t)  # RCCL over xGMI: per-doc totals + k-mer total, one collective
    tot = t.cpu().numpy()
    first = _job_first_row(res, D)
    res.set_job_totals(tot[:D].astype(np.uint64), int(tot[D]), first)
    if hasattr(model, "_get_svm"):  # ProbabilisticFilterSVMModel: label from the job's totals
        out = [None]
        if rank == 0:
            features = [[v for _, v in sorted(res.get_total_scores().items())]]
            out[0] = str(model._get_svm(exclude_ids).predict(features)[0])
        dist.broadcast_object_list(out, src=0)
        res.prediction = out[0]
    res.input_source = input_file.name
    res.save(shard_path(output_path, rank, world))
    return res


def merge_result_shards(paths) -> dict:
    """The single-process result dict from the JSON shards of a sharded job
    (in part order): per-read sections concatenated, the job's "total",
    prediction and fields from the shards (they agree).  Duplicate read ids
    across shards keep their first position and the last values, as the
    reference's dictionaries do."""
    out = None
    for p in paths:
        d = json.loads(Path(p).read_text(encoding="utf-8"))
        if out is None:
            out = {k: v for k, v in d.items()}
            out["hits"], out["num_kmers"] = {}, {}
            out["scores"] = {}
        total = d["scores"].pop("total")
        out["hits"].update(d["hits"])
        out["scores"].update(d["scores"])
        out["num_kmers"].update(d["num_kmers"])
        out["scores"]["total"] = total
    if out is not None:  # "total" is the last key of "scores", as get_scores() builds it
        out["scores"]["total"] = out["scores"].pop("total")
    return out


# ---------------------------------------------------------------- config 5: docs-sharded classify
def predict_docs_sharded(model, input_file: Path, step: int = 1, display_name: bool = False):
    """Config 5 (docs sharded): every rank holds a different species model (one
    genus of a multi-genus collection, its bank on this rank's GPU) and probes
    every read of the file; the per-read hit columns of all ranks are
    all-gathered into one MatrixResult over every rank's docs (labels in rank
    order), the same on every rank.

    Under RCCL each batch goes to the device once, is probed there
    (``docs_sharded_hits_device``: probe, narrow, all-gather over xGMI, widen)
    and only the gathered matrix, narrowed to the reads' count width, comes
    back.  Under gloo (CPU tests, shared-GPU rehearsal) the rows are probed
    from host buffers and gathered through the host."""
    return _predict_doc_columns(model, input_file, step, display_name, "multi-genus-docs-sharded")


def cobs_classic_docs(index_path: Path) -> int:
    """Document count of a classic COBS index, from its header (magic, u32
    version, u32 docs; the layout xs_bank_open reads)."""
    with open(index_path, "rb") as fh:
        head = fh.read(26)
    if not head.startswith(b"COBS:CLASSIC_INDEX") or len(head) < 26:
        raise ValueError(f"{index_path}: not a classic COBS index")
    return int.from_bytes(head[22:26], "little")


def doc_slice(num_docs: int, rank: int, world: int) -> tuple[int, int]:
    """Docs [lo, hi) of rank `rank` when one bank is column-split over `world`
    ranks (option b): the rows' byte columns are
    dealt out evenly, so lo and hi are multiples of 8 (hi = num_docs last)."""
    R = (num_docs + 7) // 8
    if not 0 <= rank < world or world > R:
        raise ValueError(f"a bank of {num_docs} docs ({R} row bytes) cannot be split over {world} ranks")
    return R * rank // world * 8, min(num_docs, R * (rank + 1) // world * 8)


def load_docs_slice(cls, json_path: Path, rank: int | None = None, world: int | None = None):
    """This rank's slice of ONE species model: `cls.load(json_path)` with only
    docs doc_slice(D, rank, world) of its bank on this rank's GPU (the model's
    metadata, display names and SVM stay whole)."""
    dist = _dist()
    rank = dist.get_rank() if rank is None else rank
    world = dist.get_world_size() if world is None else world
    from .util import slugify
    meta = json.loads(Path(json_path).read_text(encoding="utf-8"))  # the index lies where load() finds it
    index = Path(json_path).parent / slugify(meta["model_display_name"] + "-" + str(meta["model_type"])) / \
        "index.cobs_classic"
    return cls.load(json_path, docs=doc_slice(cobs_classic_docs(index), rank, world))


def predict_bank_sharded(model, input_file: Path, step: int = 1, display_name: bool = False):
    """Config 5 with ONE bank column-split over the ranks (each rank's model
    from load_docs_slice): every rank hashes every k-mer and reads its slice of
    each row; the gathered MatrixResult is the whole model's prediction (labels
    in doc order, the model's slug; an SVM model's label formed from the
    gathered totals, probabilistic_filter_svm_model.py:175-223)."""
    res = _predict_doc_columns(model, input_file, step, display_name, model.slug())
    if hasattr(model, "_get_svm") and len(res.ids):
        res.prediction = str(model._get_svm(None).predict([[v for _, v in sorted(res.get_total_scores().items())]])[0])
    return res


def _predict_doc_columns(model, input_file: Path, step: int, display_name: bool, slug: str):
    import torch
    from .bank import narrowest_count_dtype
    from .file_io import check_input_path, file_reader_device, read_batches
    from .result import MatrixResult

    dist = _dist()
    world = dist.get_world_size()
    input_file = Path(input_file)
    check_input_path(input_file)
    labels_all: list = [None] * world
    dist.all_gather_object(labels_all, model._labels(display_name))
    labels = [lab for part in labels_all for lab in part]
    on_device = collective_device().type == "cuda"
    ids, hits, nks = [], [], []
    rdev = file_reader_device(model.index) if on_device else None  # text straight to HBM
    for batch in read_batches(input_file, device=rdev):
        L = batch.lengths()
        if (L <= model.k).any():
            raise ValueError("Invalid sequence, must be longer than k")
        mx = int(((L - model.k) // step + 1).max()) if batch.n else 0
        if on_device:
            if rdev is not None:
                batch.check_valid()
                d_seq, nbytes, d_off = batch.seqs_ptr, batch.seq_bytes, batch.offsets_ptr
            else:
                pr = batch.packed
                dev = torch.device("cuda", model.index.info.device)
                d_seq = torch.from_numpy(pr.buf[:max(pr.nbytes, 1)]).to(dev)
                d_off = torch.from_numpy(pr.offsets.view(np.int64)).to(dev)
                nbytes = pr.nbytes
            g, d_nk = docs_sharded_hits_device(model.index, d_seq, nbytes, d_off, batch.n, step)
            dt = narrowest_count_dtype(mx)
            h = g.to({np.uint8: torch.uint8, np.uint16: torch.int16}.get(dt, torch.int32)).cpu().numpy()
            h = h.view(np.uint16) if dt == np.uint16 else h.view(np.uint8) if dt == np.uint8 else h.view(np.uint32)
            nk = d_nk.cpu().numpy().view(np.uint64)
        else:
            hl, nk = model._query(batch.packed, step)
            t = torch.from_numpy(np.ascontiguousarray(hl).astype(np.int32))
            h = gather_doc_shards(t, mx).numpy().view(np.uint32)  # every rank reads the same batches
        ids.append(batch.ids_packed())
        hits.append(h)
        nks.append(nk)
    ids = PackedIds.concat(ids) if ids else []
    D = len(labels)
    if hits:
        dt = max((h.dtype for h in hits), key=lambda t: t.itemsize)
        hm = np.concatenate([h.astype(dt, copy=False) for h in hits]) if len(hits) > 1 else hits[0]
        nk = np.concatenate(nks)
    else:
        hm, nk = np.zeros((0, D), np.uint8), np.zeros(0, np.uint64)
    res = MatrixResult(slug, ids, labels, hm, nk, sparse_sampling_step=step)
    res.input_source = input_file.name
    return res
