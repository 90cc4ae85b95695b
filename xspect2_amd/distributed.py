"""Multi-GPU probe: one process per GPU, torch.distributed (RCCL on ROCm).

Two partitionings:

* **reads sharded, bank replicated** (config 3) — each rank probes a
  contiguous slice of the reads against its own replica of the bank; the only
  exchange is one all-reduce (sum) of D+1 uint64 counters (per-doc totals and
  the k-mer total), the inputs of ``ModelResult.get_scores()["total"]`` and
  the SVM vector.  Per-read hit rows stay on the rank that computed them.
* **docs sharded** (config 5) — each rank holds a different bank (e.g. one
  genus of a multi-genus collection) and probes all reads; per-read hit
  vectors are all-gathered along the doc axis.

The per-rank compute is a callable so the collectives can be exercised with
``gloo`` on CPU (tests) and with the HIP banks + RCCL on MI355X.
"""
from __future__ import annotations

from typing import Callable

import numpy as np

from .packing import PackedReads


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


def allreduce_totals(totals: np.ndarray, total_kmers: int, device=None) -> tuple[np.ndarray, int]:
    """Sum of (per-doc totals, k-mer total) over all ranks (one collective)."""
    import torch
    dist = _dist()
    t = torch.from_numpy(np.concatenate([totals.astype(np.int64), [np.int64(total_kmers)]]))
    if device is not None:
        t = t.to(device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
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


def docs_sharded_hits(reads: PackedReads, step: int,
                      local_query: Callable[[PackedReads, int], tuple[np.ndarray, np.ndarray]],
                      device=None) -> tuple[np.ndarray, np.ndarray]:
    """Config 5: each rank's bank covers its own docs; gather [n, sum(D_r)] in rank order.

    The hit rows travel in the narrowest integer type that holds the largest
    k-mer count of any read on any rank (agreed by one all-reduce), and are
    widened back to uint32 on arrival."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    hits, nk = local_query(reads, step)
    n, d_local = hits.shape
    nk = np.asarray(nk)
    meta = torch.tensor([d_local, int(nk.max()) if nk.size else 0], dtype=torch.int64)
    dims = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    if device is not None:
        dims = [x.to(device) for x in dims]
        meta = meta.to(device)
    dist.all_gather(dims, meta)
    d_max = max(int(x[0].item()) for x in dims)
    dt = transport_dtype(max(int(x[1].item()) for x in dims))
    pad = torch.zeros((n, d_max), dtype=dt)
    pad[:, :d_local] = torch.from_numpy(hits.astype(np.int64)).to(dt)
    if device is not None:
        pad = pad.to(device)
    # gloo and RCCL gather no int16: 2-byte rows travel as float16 bit patterns
    # (an all-gather copies bits, it does no arithmetic)
    wire = pad.view(torch.float16) if dt == torch.int16 else pad
    parts = [torch.empty_like(wire) for _ in range(world)]
    dist.all_gather(parts, wire)
    if dt == torch.int16:
        parts = [p.view(torch.int16) for p in parts]
    cols = [p.cpu().to(torch.int64).numpy()[:, :int(d[0].item())] for p, d in zip(parts, dims)]
    return np.concatenate(cols, axis=1).astype(np.uint32), nk


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
