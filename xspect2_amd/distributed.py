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


_EXC_TYPES = {"ValueError": ValueError, "IndexError": IndexError, "KeyError": KeyError,
              "FileNotFoundError": FileNotFoundError, "NotImplementedError": NotImplementedError}


def agree_or_raise(exc: BaseException | None) -> None:
    """Every rank calls this with the exception its local step raised (or
    None) before the job's next collective.  If any rank failed, every rank
    raises: the failing rank its own exception, the others the same type and
    message as the lowest failing rank's (a rank that raised alone would
    leave its peers blocked in the next collective)."""
    dist = _dist()
    msgs: list = [None] * dist.get_world_size()
    dist.all_gather_object(msgs, None if exc is None else (type(exc).__name__, str(exc)))
    bad = [(r, m) for r, m in enumerate(msgs) if m is not None]
    if not bad:
        return
    if exc is not None:
        raise exc
    _, (tname, msg) = bad[0]
    raise _EXC_TYPES.get(tname, RuntimeError)(msg)


def alltoallv(chunks: list):
    """chunks[q] (tensors of equal trailing shape and dtype, any row count) to
    rank q; returns the list of what every rank sent this one, in rank order,
    on the collective device.  Two all_to_all_single calls: the row counts,
    then the rows."""
    import torch
    dist = _dist()
    dev = collective_device()
    sizes = [int(c.shape[0]) for c in chunks]
    cnt = torch.tensor(sizes, dtype=torch.int64, device=dev)
    rcnt = torch.empty_like(cnt)
    dist.all_to_all_single(rcnt, cnt)
    rs = [int(x) for x in rcnt.tolist()]
    send = torch.cat([c.to(dev) for c in chunks]).contiguous()
    recv = torch.empty((sum(rs), *send.shape[1:]), dtype=send.dtype, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=rs, input_split_sizes=sizes)
    return list(torch.split(recv, rs))


def _dup_messages(t: np.ndarray, world: int) -> list[np.ndarray]:
    """The owner's instructions for its candidate records ``t`` (rows of
    (key0, key1, source rank, source index)): for every key held by more than
    one record, the record first in file order (rank, then index) keeps the id
    and takes the values of the last, every other record drops it.  Returns,
    per destination rank, rows (kind, index, src rank, src index): kind 0 =
    keep, values from (src rank, src index); kind 1 = drop.  Vectorised: one
    lexsort over the candidates, no per-group loop."""
    out = [np.zeros((0, 4), np.int64) for _ in range(world)]
    if t.shape[0] < 2:
        return out
    a = t[np.lexsort((t[:, 3], t[:, 2], t[:, 1], t[:, 0]))]
    start = np.concatenate([[True], (a[1:, 0] != a[:-1, 0]) | (a[1:, 1] != a[:-1, 1])])
    gid = np.cumsum(start) - 1
    first = np.flatnonzero(start)
    size = np.diff(np.concatenate([first, [a.shape[0]]]))
    dup = np.flatnonzero(size > 1)
    if not dup.size:
        return out
    f, lst = a[first[dup]], a[first[dup] + size[dup] - 1]
    keep = np.stack([f[:, 2], np.zeros(dup.size, np.int64), f[:, 3], lst[:, 2], lst[:, 3]], axis=1)
    d = a[(size[gid] > 1) & ~start]
    drop = np.stack([d[:, 2], np.ones(d.shape[0], np.int64), d[:, 3], np.zeros_like(d[:, 3]),
                     np.zeros_like(d[:, 3])], axis=1)
    msgs = np.concatenate([keep, drop])
    return [np.ascontiguousarray(msgs[msgs[:, 0] == q, 1:]) for q in range(world)]


def resolve_cross_shard_duplicates(res) -> int:
    """Apply the reference's rule for repeated read ids to one shard of a
    read-sharded job (``res``: this rank's MatrixResult, its own repeats
    already collapsed): the reference keeps one dict entry per id, at the
    position of its FIRST record with the values of its LAST record
    (``hits[record.id] = ...``, probabilistic_filter_model.py:310), and sums
    the job totals over that dict (result.py:76-90).

    Ids are keyed by 128 bits (XXH64 of the id bytes with two seeds,
    xs_ids_hash128); key half 0 picks the owning rank.  Round 1 sends only
    key half 0 (8 B per read) to the owner, which finds the records whose
    half 0 another record shares (the candidates: the repeats, plus ~n^2/2^65
    accidental pairs); round 2 fetches half 1 and the read index of the
    candidates only.  For each full key held by several records, the rank
    holding the first record keeps the id at its position and takes the hit
    row and k-mer count of the last record (fetched from its rank); every
    other rank drops the id.  Merging the shards in part order then gives the
    single-process dictionaries, and each id enters the job totals once.
    Returns the number of rows this rank dropped.  Two different ids share a
    key with probability ~n^2 / 2^129."""
    import torch
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    if world == 1:
        return 0
    ids = res.ids if isinstance(res.ids, PackedIds) else PackedIds.of(res.ids)
    n = len(ids)
    key = ids.hash128().view(np.int64)                             # [n, 2]
    owner = (key[:, 0].view(np.uint64) % np.uint64(world)).astype(np.int64)
    sent = [np.flatnonzero(owner == q) for q in range(world)]      # my rows, in the order each owner gets them
    # round 1: half 0 of every key to its owner
    got = [g.cpu().numpy() for g in alltoallv([torch.from_numpy(np.ascontiguousarray(key[o, 0])) for o in sent])]
    k0 = np.concatenate(got) if got else np.zeros(0, np.int64)
    src = np.repeat(np.arange(world, dtype=np.int64), [g.shape[0] for g in got])
    pos = np.concatenate([np.arange(g.shape[0], dtype=np.int64) for g in got]) if got else np.zeros(0, np.int64)
    srt = np.sort(k0)
    shared = srt[1:][srt[1:] == srt[:-1]]                          # key halves held more than once
    cand = np.zeros(0, np.int64)
    if shared.size:                                                # their records, by source rank then position
        from ._lib import check, load
        hit = np.empty(k0.size, dtype=np.uint8)
        shared = np.ascontiguousarray(shared)
        check(load().xs_u64_member_mask(k0.ctypes.data, k0.size, shared.ctypes.data, shared.size, hit.ctypes.data))
        cand = np.flatnonzero(hit)
    # round 2: half 1 and the read index of each candidate, from its source
    req = alltoallv([torch.from_numpy(np.ascontiguousarray(pos[cand][src[cand] == q])) for q in range(world)])
    answers = []
    for r, p in enumerate(req):
        rows = sent[r][p.cpu().numpy().astype(np.int64)]
        answers.append(torch.from_numpy(np.ascontiguousarray(np.stack([key[rows, 1], rows], axis=1))))
    back1 = alltoallv(answers)
    kv = np.concatenate([b.cpu().numpy().reshape(-1, 2) for b in back1]) if back1 else np.zeros((0, 2), np.int64)
    t = np.stack([k0[cand], kv[:, 0], src[cand], kv[:, 1]], axis=1) if cand.size else np.zeros((0, 4), np.int64)
    inst = alltoallv([torch.from_numpy(m) for m in _dup_messages(t, world)])
    inst = np.concatenate([x.cpu().numpy().reshape(-1, 4) for x in inst]) if inst else np.zeros((0, 4), np.int64)
    keep_take = inst[inst[:, 0] == 0]
    drop = inst[inst[:, 0] == 1, 1]
    # fetch the last records' rows: request (their index, my index) from their rank, answer with the rows
    req = alltoallv([torch.from_numpy(np.ascontiguousarray(keep_take[keep_take[:, 2] == q][:, [3, 1]]))
                     for q in range(world)])
    D = res.hits.shape[1]
    answers = []
    for q, r in enumerate(req):
        r = r.cpu().numpy().reshape(-1, 2)
        row = np.zeros((r.shape[0], D + 2), dtype=np.int64)
        row[:, 0] = r[:, 1]
        if r.shape[0]:
            row[:, 1] = res.num_kmers[r[:, 0]].astype(np.int64)
            row[:, 2:] = res.hits[r[:, 0]].astype(np.int64)
        answers.append(torch.from_numpy(row))
    back = alltoallv(answers)
    back = np.concatenate([b.cpu().numpy().reshape(-1, D + 2) for b in back]) if back else np.zeros((0, D + 2))
    if back.shape[0]:
        need = int(back[:, 2:].max()) if D else 0
        hits = res.hits
        if need > np.iinfo(hits.dtype).max:
            hits = hits.astype(np.uint16 if need <= 0xFFFF else np.uint32)
        else:
            hits = hits.copy()
        nk = res.num_kmers.copy()
        idx = back[:, 0]
        hits[idx] = back[:, 2:].astype(hits.dtype)
        nk[idx] = back[:, 1].astype(np.uint64)
        res.hits, res.num_kmers = hits, nk
    if drop.size:
        keep = np.ones(n, dtype=bool)
        keep[drop] = False
        rows = np.flatnonzero(keep)
        res.ids = ids.drop(drop) if isinstance(res.ids, PackedIds) else [res.ids[i] for i in rows.tolist()]
        res.hits = np.ascontiguousarray(res.hits[rows])
        res.num_kmers = np.ascontiguousarray(res.num_kmers[rows])
    return int(drop.size)


def set_job_totals(res, device=None) -> None:
    """Make ``res`` (this rank's shard) carry the whole job's "total": one
    all-reduce of the D+1 counters (per-doc sums, k-mer total) on `device`
    (RCCL) or the host (gloo), and the job's first hit row, which orders the
    "total" labels as the reference's get_total_hits does (result.py:84-90)."""
    import torch
    D = len(res.labels)
    local = np.zeros(D + 1, dtype=np.int64)
    if len(res.ids):
        # a read named "misclassified" leaves the hits (result.py:43) but keeps its k-mers
        m = _misclassified_row(res)
        hits = res.hits if m is None else np.delete(res.hits, m, axis=0)
        local[:D] = hits.sum(axis=0, dtype=np.uint64).astype(np.int64)
        local[D] = int(res.num_kmers.sum())
    t = torch.from_numpy(local)
    if device is not None:
        t = t.to(device)
    allreduce_(t)  # RCCL over xGMI: per-doc totals + k-mer total, one collective
    tot = t.cpu().numpy()
    first = _job_first_row(res, D)
    res.set_job_totals(tot[:D].astype(np.uint64), int(tot[D]), first)


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


def _misclassified_row(res):
    """Row of this shard's read literally named "misclassified" (None if
    none): the reference pops it from the hits into the result's
    "misclassified" field (result.py:43)."""
    ids = res.ids
    if "misclassified" not in ids:
        return None
    return ids.index("misclassified")


def _job_first_row(res, D: int) -> np.ndarray:
    """Hit row of the job's first read (first read of the lowest rank that has
    one, a read named "misclassified" excepted: it is not in the reference's
    hits), which orders the labels of the job's "total" scores as the
    reference's get_total_hits does (result.py:84-90)."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    m = _misclassified_row(res)
    first = 0 if m != 0 else 1  # the first row that is in the hits
    have = len(res.ids) - (m is not None)
    flags = [torch.zeros(1, dtype=torch.int64, device=collective_device()) for _ in range(world)]
    dist.all_gather(flags, _on_wire(torch.tensor([have], dtype=torch.int64)))
    owners = [r for r, f in enumerate(flags) if int(f.item()) > 0]
    if not owners:
        raise IndexError("list index out of range")  # get_total_hits on no reads, as the reference
    row = torch.zeros(D, dtype=torch.int64)
    if dist.get_rank() == owners[0]:
        row = torch.from_numpy(res.hits[first].astype(np.int64))
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
    A read id repeated in different shards follows the reference's dict
    (``resolve_cross_shard_duplicates``): one entry, at the first record's
    position with the last record's values, counted once in the totals.
    An error on any rank (a read no longer than k, a malformed record)
    raises on every rank.  Returns this rank's MatrixResult (a shard)."""
    import torch
    from .file_io import FileShard
    from .probabilistic_filter_model import ProbabilisticFilterModel

    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    input_file = Path(input_file)
    res, err = None, None
    try:
        res = ProbabilisticFilterModel.predict_columnar(model, FileShard(input_file, rank, world), exclude_ids,
                                                        step, display_name)
    except Exception as e:  # noqa: BLE001 - re-raised on every rank by agree_or_raise
        err = e
    agree_or_raise(err)
    resolve_cross_shard_duplicates(res)
    dev = torch.device("cuda", model.index.info.device) if collective_device().type == "cuda" else None
    set_job_totals(res, dev)
    _svm_label(model, res, exclude_ids)
    res.input_source = input_file.name
    res.save(shard_path(output_path, rank, world))
    return res


def _svm_label(model, res, exclude_ids=None) -> None:
    """SVM models (ProbabilisticFilterSVMModel, probabilistic_filter_svm_model.py:
    175-223): rank 0 classifies the job's total scores, every rank gets the label."""
    if not hasattr(model, "_get_svm"):
        return
    dist = _dist()
    out = [None]
    if dist.get_rank() == 0:
        features = [[v for _, v in sorted(res.get_total_scores().items())]]
        out[0] = str(model._get_svm(exclude_ids).predict(features)[0])
    dist.broadcast_object_list(out, src=0)
    res.prediction = out[0]


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
        if d.get("misclassified") is not None:  # the shard that held the read named so (result.py:43)
            out["misclassified"] = d["misclassified"]
        out["hits"].update(d["hits"])
        out["scores"].update(d["scores"])
        out["num_kmers"].update(d["num_kmers"])
        out["scores"]["total"] = total
    if out is not None:  # "total" is the last key of "scores", as get_scores() builds it
        out["scores"]["total"] = out["scores"].pop("total")
    return out


def _json_members(buf, key: bytes, next_key: bytes) -> tuple[int, int]:
    """Byte range of the members inside the top-level object `key` of a
    result file (ModelResult.save layout, indent 4), empty for ``{}``."""
    a = buf.find(b'\n    "' + key + b'": ')
    b = buf.find(b',\n    "' + next_key + b'": ', a)
    if a < 0 or b < 0:
        raise ValueError(f"not a result file: no {key.decode()!r} section")
    a += len(key) + 9
    if buf[a:b] == b"{}":
        return a, a
    return a + 2, b - 6  # inside "{\n" ... "\n    }"


def merge_result_files(paths, out_path: Path) -> None:
    """Stream the JSON shards of a sharded job (in part order) into the
    single-process JSON file, byte for byte, without parsing them: each
    read's sections are already in its shard in the reference's dict order
    (``resolve_cross_shard_duplicates`` leaves every id in the shard of its
    first record), so the merged file is the shards' per-read members
    concatenated, with the job's "total", prediction and fields of the first
    shard (all shards carry the same).  Memory stays bounded by the mapped
    files; for the dict form use ``merge_result_shards``."""
    import mmap
    files, maps = [], []
    try:
        for p in paths:
            fh = open(p, "rb")
            files.append(fh)
            maps.append(mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ) if Path(p).stat().st_size else b"")
        parts = []
        for m in maps:
            h = _json_members(m, b"hits", b"scores")
            s = _json_members(m, b"scores", b"num_kmers")
            n = _json_members(m, b"num_kmers", b"misclassified")
            t = m.rfind(b'\n        "total": ', s[0] - 1, s[1])
            total = (t + 1, s[1])
            before = (s[0], t - 1) if t > s[0] else (s[0], s[0])  # members before "total" (no trailing ",")
            parts.append((h, before, total, n))
        m0, (h0, _, total0, _) = maps[0], parts[0]

        def members(out, which):
            first = True
            for m, pr in zip(maps, parts):
                a, b = pr[which]
                if b > a:
                    out.write(b"" if first else b",\n")
                    out.write(m[a:b])
                    first = False
            return not first

        with open(out_path, "wb") as out:
            out.write(m0[:h0[0] - (2 if h0[1] > h0[0] else 0)])  # up to `"hits": `
            if any(pr[0][1] > pr[0][0] for pr in parts):
                out.write(b"{\n")
                members(out, 0)
                out.write(b"\n    }")
            else:
                out.write(b"{}")
            out.write(b',\n    "scores": {\n')
            if members(out, 1):
                out.write(b",\n")
            out.write(m0[total0[0]:total0[1]])
            out.write(b'\n    },\n    "num_kmers": ')
            if any(pr[3][1] > pr[3][0] for pr in parts):
                out.write(b"{\n")
                members(out, 3)
                out.write(b"\n    }")
            else:
                out.write(b"{}")
            # the "misclassified" section of the shard that held such a read (result.py:43), else shard 0's
            tails = [m[m.find(b',\n    "misclassified": '):] for m in maps]
            tail = tails[0]
            for t in tails:
                if not t.startswith(b',\n    "misclassified": null'):
                    mis = t[:t.find(b',\n    "input_source": ')]
                    tail = mis + tails[0][tails[0].find(b',\n    "input_source": '):]
                    break
            out.write(tail)
    finally:
        for m in maps:
            if isinstance(m, mmap.mmap):
                m.close()
        for fh in files:
            fh.close()


# ---------------------------------------------------------------- config 5: docs-sharded classify
def predict_docs_sharded(model, input_file: Path, step: int = 1, display_name: bool = False):
    """Config 5 (docs sharded): every rank holds a different species model (one
    genus of a multi-genus collection, its bank on this rank's GPU).  Rank r
    parses only part r of the file (record-aligned byte ranges, as config 3);
    each batch's reads are all-gathered, every rank probes every rank's reads
    against its bank, and the hit columns go back to the rank that owns the
    reads (``exchange_doc_columns``: one all-to-all in the narrowest exact
    integer type).  Returns this rank's shard: its own reads with the hit
    columns of every rank's docs (labels in rank order), and the job's
    "total" over all reads (``set_job_totals``).  ``merge_result_shards`` of
    the saved shards (``classify_docs_sharded``) is the JSON one process
    probing every bank writes.  Under RCCL reads and hits stay on the device
    from the reader to the exchanged columns; under gloo (CPU tests, the
    shared-GPU rehearsal) they go through host tensors."""
    return _predict_doc_columns(model, input_file, step, display_name, "multi-genus-docs-sharded")


def classify_docs_sharded(model, input_file: Path, output_path: Path, step: int = 1, display_name: bool = False):
    """Config 5 for one input file: ``predict_docs_sharded`` and every rank
    writes its JSON shard (``shard_path``), as ``classify_species_sharded``
    does for config 3 (the reference writes one result per input,
    src/xspect/classify.py:43-92, src/xspect/models/result.py:178-189)."""
    dist = _dist()
    res = predict_docs_sharded(model, input_file, step, display_name)
    res.save(shard_path(output_path, dist.get_rank(), dist.get_world_size()))
    return res


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
    each row; the result is this rank's shard of the whole model's prediction
    (its own reads, labels in doc order, the model's slug, the job's totals);
    an SVM model's label is formed on rank 0 from the job's total scores
    (probabilistic_filter_svm_model.py:175-223) and broadcast."""
    res = _predict_doc_columns(model, input_file, step, display_name, model.slug())
    _svm_label(model, res)
    return res


def exchange_doc_columns(hits, counts: list[int], dims: list[int], wire):
    """Hit columns [sum(counts), D_r] of this rank (rows: rank 0's reads, then
    rank 1's, ...) -> this rank's reads with every rank's columns
    [counts[rank], sum(dims)] in the wire dtype (uint8 / int16 / int32, from
    ``transport_dtype``), on the tensor's device.  Rows are narrowed where
    they are, padded to the widest D_r and sent by one all-to-all (RCCL over
    xGMI on the device); the narrow result is what the shard keeps."""
    import torch
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    d_local, d_max = int(hits.shape[1]), max(dims)
    if dims[rank] != d_local or int(hits.shape[0]) != sum(counts):
        raise ValueError("hit columns do not match the agreed layout")
    n_me = counts[rank]
    if d_local == d_max:
        send = hits.to(wire)  # lossless: counts <= k-mers per read <= the wire type's maximum
    else:
        send = torch.zeros((hits.shape[0], d_max), dtype=wire, device=hits.device)
        send[:, :d_local] = hits.to(wire)
    # gloo and RCCL move no int16: 2-byte rows travel as float16 bit patterns
    wire_view = send.view(torch.float16) if wire == torch.int16 else send
    w = _on_wire(wire_view.contiguous())
    recv = torch.empty((world * n_me, d_max), dtype=w.dtype, device=w.device)
    dist.all_to_all_single(recv, w, output_split_sizes=[n_me] * world, input_split_sizes=list(counts))
    if wire == torch.int16:
        recv = recv.view(torch.int16)
    recv = recv.to(hits.device) if recv.device != hits.device else recv
    blocks = recv.view(world, n_me, d_max)
    return torch.cat([blocks[r, :, :dims[r]] for r in range(world)], dim=1).contiguous()


def _read_device_batch(batch, dev, pad_to: int):
    """A device reader batch's sequences and offsets as torch tensors on `dev`
    (sequences padded to `pad_to` bytes for the all-gather)."""
    import torch
    from ._lib import check, load
    seq = torch.zeros(max(pad_to, 1), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    if batch.seq_bytes:
        check(load().xs_memcpy_device(seq.data_ptr(), batch.seqs_ptr, batch.seq_bytes, stream))
    off = torch.from_numpy(batch.offsets.view(np.int64)).to(dev)
    return seq, off


def _predict_doc_columns(model, input_file: Path, step: int, display_name: bool, slug: str):
    import torch
    from .file_io import check_input_path, file_reader_device, read_batches
    from .packing import PackedReads
    from .result import MatrixResult

    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    input_file = Path(input_file)
    err = None
    try:
        check_input_path(input_file)
        if step < 1:
            raise ValueError("step must be >= 1")
    except Exception as e:  # noqa: BLE001 - raised on every rank below
        err = e
    agree_or_raise(err)
    # the layout, once per file: every rank's labels (doc columns) and k
    meta_all: list = [None] * world
    dist.all_gather_object(meta_all, (model._labels(display_name), int(model.k)))
    labels = [lab for part, _ in meta_all for lab in part]
    dims = [len(part) for part, _ in meta_all]
    ks = {k for _, k in meta_all}
    if len(ks) != 1:
        raise ValueError(f"docs-sharded models must share k (one k-mer count per read), got {sorted(ks)}")
    k = ks.pop()
    on_device = collective_device().type == "cuda"
    dev = torch.device("cuda", model.index.info.device) if on_device else torch.device("cpu")
    rdev = file_reader_device(model.index) if on_device else None
    ids, hits, nks = [], [], []
    batches = read_batches(input_file, part=rank, parts=world, device=rdev)
    try:
        while True:
            b, err = None, None
            try:
                b = next(batches, None)
                if b is not None and rdev is not None:
                    b.check_valid()
                L = b.lengths() if b is not None and b.n else np.zeros(0, dtype=np.uint64)
                if (L <= k).any():
                    raise ValueError("Invalid sequence, must be longer than k")
            except Exception as e:  # noqa: BLE001 - raised on every rank
                err = e
            agree_or_raise(err)
            n = b.n if b is not None else 0
            nbytes = (b.seq_bytes if rdev is not None else b.packed.nbytes) if n else 0
            m = torch.tensor([n, nbytes, int(L.max()) if n else 0], dtype=torch.int64, device=dev)
            allm = [torch.empty_like(m) for _ in range(world)]
            dist.all_gather(allm, m)
            meta = torch.stack(allm).cpu().numpy()
            counts, sizes = meta[:, 0].tolist(), meta[:, 1].tolist()
            if sum(counts) == 0:
                break
            wire = transport_dtype((int(meta[:, 2].max()) - k) // step + 1)
            b_max, n_max = max(max(sizes), 1), max(counts)
            # every rank's reads of this batch, on every rank
            if rdev is not None and n:
                seq, off = _read_device_batch(b, dev, b_max)
            else:
                seq = torch.zeros(b_max, dtype=torch.uint8)
                off = torch.zeros(n + 1, dtype=torch.int64)
                if n:
                    seq[:nbytes] = torch.from_numpy(b.packed.buf[:nbytes])
                    off = torch.from_numpy(b.packed.offsets.astype(np.int64))
                seq, off = seq.to(dev), off.to(dev)
            offp = torch.zeros(n_max + 1, dtype=torch.int64, device=dev)
            offp[:n + 1] = off[:n + 1]
            seqs = [torch.empty_like(seq) for _ in range(world)]
            offs = [torch.empty_like(offp) for _ in range(world)]
            dist.all_gather(seqs, seq)
            dist.all_gather(offs, offp)
            cat_seq = torch.cat([seqs[q][:sizes[q]] for q in range(world)] or [seq[:0]])
            base = np.concatenate([[0], np.cumsum(sizes)]).tolist()
            cat_off = torch.cat([offs[q][:counts[q]] + base[q] for q in range(world)] +
                                [torch.tensor([base[-1]], dtype=torch.int64, device=dev)])
            N = sum(counts)
            lo = int(np.sum(counts[:rank]))
            # the probe of every rank's reads (it allocates N x D_r counts): a failure on one
            # rank raises on every rank before the exchange, instead of leaving the others in it
            err = None
            try:
                if on_device:
                    d_hits = torch.empty((N, model.index.num_docs), dtype=torch.int32, device=dev)
                    d_nk = torch.empty(N, dtype=torch.int64, device=dev)
                    stream = torch.cuda.current_stream(dev)
                    model.index.query_device(cat_seq, base[-1], cat_off, N, step, d_hits, d_nk, None,
                                             stream=stream.cuda_stream)
                    stream.synchronize()
                    local = d_hits
                    nk = d_nk[lo:lo + n].cpu().numpy().view(np.uint64)
                else:
                    buf = np.concatenate([cat_seq.numpy(), np.zeros(1, dtype=np.uint8)])
                    h, nk_all = model._query(PackedReads(buf, cat_off.numpy().astype(np.uint64)), step)
                    local = torch.from_numpy(np.ascontiguousarray(h).astype(np.int32))
                    nk = np.asarray(nk_all, dtype=np.uint64)[lo:lo + n]
            except Exception as e:  # noqa: BLE001 - raised on every rank by agree_or_raise
                err = e
            agree_or_raise(err)
            cols = exchange_doc_columns(local, counts, dims, wire)
            hc = cols.cpu().numpy()
            hc = hc.view(np.uint16) if wire == torch.int16 else hc.view(np.uint32) if wire == torch.int32 else hc
            if n:
                ids.append(b.ids_packed())
                hits.append(hc)
                nks.append(nk)
    finally:
        batches.close()
    D = len(labels)
    res, err = None, None
    try:
        if hits:
            dt = max((h.dtype for h in hits), key=lambda t: t.itemsize)
            hm = np.concatenate([h.astype(dt, copy=False) for h in hits]) if len(hits) > 1 else hits[0]
            nk = np.concatenate(nks)
        else:
            hm, nk = np.zeros((0, D), np.uint8), np.zeros(0, np.uint64)
        res = MatrixResult(slug, PackedIds.concat(ids) if ids else [], labels, hm, nk, sparse_sampling_step=step)
    except Exception as e:  # noqa: BLE001 - raised on every rank by agree_or_raise
        err = e
    agree_or_raise(err)
    resolve_cross_shard_duplicates(res)
    set_job_totals(res, dev if on_device else None)
    res.input_source = input_file.name
    return res
