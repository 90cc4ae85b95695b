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


def docs_sharded_hits(reads: PackedReads, step: int,
                      local_query: Callable[[PackedReads, int], tuple[np.ndarray, np.ndarray]],
                      device=None) -> tuple[np.ndarray, np.ndarray]:
    """Config 5: each rank's bank covers its own docs; gather [n, sum(D_r)] in rank order."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    hits, nk = local_query(reads, step)
    n, d_local = hits.shape
    dims = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    mine = torch.tensor([d_local], dtype=torch.int64)
    if device is not None:
        dims = [x.to(device) for x in dims]
        mine = mine.to(device)
    dist.all_gather(dims, mine)
    d_max = max(int(x.item()) for x in dims)
    pad = np.zeros((n, d_max), dtype=np.int32)
    pad[:, :d_local] = hits.view(np.int32)
    t = torch.from_numpy(pad)
    if device is not None:
        t = t.to(device)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    cols = [p.cpu().numpy()[:, :int(d.item())] for p, d in zip(parts, dims)]
    return np.concatenate(cols, axis=1).view(np.uint32), np.asarray(nk)


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
