"""Device-resident filter banks (COBS classic / compact, rbloom) behind the C ABI.

A :class:`Bank` owns one ``xs_bank`` handle: the bank image lives in HBM for
the lifetime of the object (reference: ``cobs.Search(path, True)`` at
``src/xspect/models/probabilistic_filter_model.py:389`` keeps it in host RAM
and is re-entered once per read).
"""
from __future__ import annotations

import ctypes
import math
from pathlib import Path
from typing import Iterable, Sequence

import numpy as np

from . import _lib
from ._lib import (XS_BANK_COBS_CLASSIC, XS_BANK_COBS_COMPACT, XS_BANK_RBLOOM, BankInfo,
                   check, load)
from .packing import PackedReads, pack_sequences

KIND_NAMES = {XS_BANK_COBS_CLASSIC: "cobs_classic", XS_BANK_COBS_COMPACT: "cobs_compact",
              XS_BANK_RBLOOM: "rbloom"}


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a is not None and a.size else 0


def cobs_signature_size(num_terms: int, num_hashes: int, fpr: float) -> int:
    """COBS calc_signature_size (restated): ceil(-h*n / ln(1 - fpr^(1/h)))."""
    return int(math.ceil(-num_hashes * num_terms / math.log(1.0 - math.pow(fpr, 1.0 / num_hashes))))


def bloom_parameters(expected_items: int, fpr: float) -> tuple[int, int]:
    """(nbytes, K) of rbloom.Bloom(expected_items, fpr) (restated, unverified)."""
    if expected_items <= 0 or not 0.0 < fpr < 1.0:
        raise ValueError("expected_items must be > 0 and 0 < fpr < 1")
    size_bits = int(-expected_items * math.log(fpr) / (math.log(2) ** 2))
    nhash = max(1, math.ceil(size_bits / expected_items * math.log(2)))
    return (max(size_bits, 1) + 7) // 8, nhash


def _device_batch(reads) -> bool:
    """A device-mode reader batch (file_io.DeviceSeqBatch): reads in HBM."""
    return hasattr(reads, "seqs_ptr")


def _kmers_of(length: int, k: int, step: int) -> int:
    return (length - k) // step + 1 if length >= k else 0


def max_kmers(reads: PackedReads, k: int, step: int) -> int:
    """Largest sampled k-mer count ceil((len - k + 1) / step) of a batch."""
    if reads.n == 0:
        return 0
    L = int(np.diff(reads.offsets).max())
    return (L - k) // step + 1 if L >= k else 0


def narrowest_count_dtype(max_count: int):
    """uint8 / uint16 / uint32: the narrowest type that holds counts up to max_count."""
    return np.uint8 if max_count <= 0xFF else np.uint16 if max_count <= 0xFFFF else np.uint32


class _PinnedAlloc:
    """Page-locked host memory from xs_host_alloc, freed with the last array view."""

    def __init__(self, nbytes: int):
        p = ctypes.c_void_p()
        check(load().xs_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.__array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (self.ptr, False),
                                    "version": 3}

    def __del__(self):
        try:
            load().xs_host_free(self.ptr)
        except Exception:  # pragma: no cover - interpreter shutdown order
            pass


def pinned_empty(shape, dtype=np.uint32) -> np.ndarray:
    """An uninitialised array in pinned host memory (reuse it as ``out=`` of
    ``Bank.query``: results arrive by DMA, without first-touch page faults)."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    return np.asarray(_PinnedAlloc(max(n, 1)))[:n].view(dtype).reshape(shape)


class _HostPool:
    """Recycled pageable host blocks for the arrays Bank.query returns.

    A fresh pageable array costs its pages twice: faulting them in on the
    first write (cheap inside the call now: the copy-out's eight threads take
    2 MiB pages, +0.5 ms per 400 MB) and unmapping them when the caller drops
    the array (14-23 ms per 400 MB on the MI355X boxes, more than the query's
    17 ms; profiles/r05m_fresh_out.json).  So result arrays are views of
    blocks kept here; a block goes back into service once no array refers to
    it any more (every numpy view of a block holds the block itself as its
    base, so the block's reference count says whether one is alive), and a
    repeated query of the same size writes into pages faulted once.  A block's
    count is compared with the count it had when it was appended, measured
    the same way, so the test does not depend on how the interpreter counts
    getrefcount's own argument.  Consumers must hold the arrays (or views of
    them), not only their buffer address.  At most ``cap`` bytes are kept
    (2 GiB: config 2's 400 MB uint32 matrix and a few batches' rows); larger
    requests get fresh arrays, and release_host_memory() gives the free blocks
    back."""

    def __init__(self, cap: int = 2 << 30, min_bytes: int = 8 << 20):
        import sys
        import threading
        self._refs = sys.getrefcount
        self._lock = threading.Lock()  # queries from several threads (the reference's web workers)
        self.blocks: list[np.ndarray] = []
        self._base: list[int] = []  # each block's reference count with no array of it alive
        self.cap, self.min_bytes = cap, min_bytes

    def _free(self, i: int) -> bool:
        return self._refs(self.blocks[i]) <= self._base[i]

    def _pop(self, i: int) -> int:
        self._base.pop(i)
        return self.blocks.pop(i).size

    def empty(self, shape, dtype) -> np.ndarray:
        dtype = np.dtype(dtype)
        n = int(np.prod(shape)) * dtype.itemsize
        if n < self.min_bytes:
            return np.empty(shape, dtype)
        with self._lock:  # a block is checked free and handed out in one step
            return self._take(n, shape, dtype)

    def _take(self, n: int, shape, dtype) -> np.ndarray:
        for i in range(len(self.blocks)):
            if n <= self.blocks[i].size <= 2 * n and self._free(i):
                return self.blocks[i][:n].view(dtype).reshape(shape)
        kept = sum(b.size for b in self.blocks)
        i = 0
        while kept + n > self.cap and i < len(self.blocks):  # drop free blocks, oldest first
            if self._free(i):
                kept -= self._pop(i)
            else:
                i += 1
        if kept + n > self.cap:
            return np.empty(shape, dtype)
        self.blocks.append(np.empty(n, np.uint8))
        self._base.append(self._refs(self.blocks[-1]))  # measured as _free measures it, no view yet
        return self.blocks[-1][:n].view(dtype).reshape(shape)


    def release(self) -> int:
        """Forget every block no array refers to any more; returns the bytes let go."""
        with self._lock:
            freed, i = 0, 0
            while i < len(self.blocks):
                if self._free(i):
                    freed += self._pop(i)
                else:
                    i += 1
            return freed


_HOST_POOL = _HostPool()


def release_host_memory() -> int:
    """Give back the host blocks ``Bank.query`` keeps for reuse (those no
    result array still uses); returns the bytes released."""
    return _HOST_POOL.release()


class Bank:
    """One filter bank resident on one GPU."""

    def __init__(self, handle: ctypes.c_void_p):
        self._h = handle
        self._names: list[str] | None = None

    # ------------------------------------------------------------ creation
    @classmethod
    def open(cls, path: str | Path, kind: int, device: int = 0, term_size: int | None = None,
             docs: tuple[int, int] | None = None) -> "Bank":
        """Load an index file.  docs=(lo, hi): a classic COBS index with only
        docs [lo, hi) resident (lo, hi multiples of 8 or hi = the doc count):
        one rank's column slice of a docs-sharded bank (xs_bank_open_docs)."""
        path = Path(path)
        if not path.exists():
            raise FileNotFoundError(f"Index file not found at {path}")
        h = ctypes.c_void_p()
        if docs is not None:
            if kind != XS_BANK_COBS_CLASSIC:
                raise ValueError("only classic COBS banks open as doc slices")
            check(load().xs_bank_open_docs(str(path).encode(), device, int(docs[0]), int(docs[1]), ctypes.byref(h)))
            return cls(h)
        check(load().xs_bank_open(str(path).encode(), kind, device, ctypes.byref(h)))
        bank = cls(h)
        if kind == XS_BANK_RBLOOM and term_size is not None:
            check(load().xs_bank_set_term_size(h, term_size))
        return bank

    @classmethod
    def create_cobs(cls, term_size: int, num_hashes: int, signature_sizes: Sequence[int],
                    num_docs: int, doc_names: Sequence[str] | None = None,
                    page_size: int | None = None, compact: bool = False,
                    device: int = 0) -> "Bank":
        if compact:
            if page_size is None:
                raise ValueError("compact banks need a page size")
            kind = XS_BANK_COBS_COMPACT
        else:
            kind = XS_BANK_COBS_CLASSIC
            page_size = (num_docs + 7) // 8
        sig = np.ascontiguousarray(signature_sizes, dtype=np.uint64)
        names_arr = None
        keep = []
        if doc_names is not None:
            if len(doc_names) != num_docs:
                raise ValueError("doc_names must have num_docs entries")
            keep = [n.encode() for n in doc_names]
            names_arr = (ctypes.c_char_p * num_docs)(*keep)
        h = ctypes.c_void_p()
        check(load().xs_bank_create_cobs(device, kind, term_size, num_hashes, num_docs, page_size,
                                         len(sig), _ptr(sig),
                                         ctypes.cast(names_arr, ctypes.c_void_p) if names_arr else None,
                                         ctypes.byref(h)))
        return cls(h)

    @classmethod
    def create_bloom(cls, term_size: int, nbytes: int, num_hashes: int, device: int = 0) -> "Bank":
        h = ctypes.c_void_p()
        check(load().xs_bank_create_bloom(device, term_size, nbytes, num_hashes, ctypes.byref(h)))
        return cls(h)

    # ------------------------------------------------------------ properties
    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise ValueError("bank is closed")
        return self._h

    @property
    def info(self) -> BankInfo:
        inf = BankInfo()
        check(load().xs_bank_info(self.handle, ctypes.byref(inf)))
        return inf

    @property
    def kind(self) -> int:
        return self.info.kind

    @property
    def device(self) -> int:
        return int(self.info.device)

    @property
    def num_docs(self) -> int:
        return int(self.info.num_docs)

    @property
    def term_size(self) -> int:
        return int(self.info.term_size)

    @property
    def doc_names(self) -> list[str]:
        if self._names is None:
            lib = load()
            self._names = [lib.xs_bank_doc_name(self.handle, i).decode() for i in range(self.num_docs)]
        return self._names

    def signature_sizes(self) -> list[int]:
        """Rows of every doc group (COBS banks)."""
        g = int(self.info.num_groups)
        out = np.zeros(g, dtype=np.uint64)
        check(load().xs_bank_signature_sizes(self.handle, _ptr(out), g))
        return [int(x) for x in out]

    def payload_bytes(self) -> int:
        inf = self.info
        if inf.kind == XS_BANK_RBLOOM:
            return int(inf.bloom_bits // 8)
        return int(inf.signature_rows * inf.page_size)

    # ------------------------------------------------------------ building
    def build(self, reads: PackedReads | Iterable, docs: Sequence[int] | np.ndarray | None = None) -> None:
        pr = reads if isinstance(reads, PackedReads) else pack_sequences(reads)
        d = None
        if self.kind != XS_BANK_RBLOOM:
            if docs is None:
                raise ValueError("COBS banks need the doc index of every record")
            d = np.ascontiguousarray(docs, dtype=np.uint32)
            if d.size != pr.n:
                raise ValueError("one doc index per record")
        check(load().xs_bank_build(self.handle, _ptr(pr.buf), _ptr(pr.offsets), _ptr(d) if d is not None else None, pr.n))

    def build_device(self, seqs, seq_bytes: int, offsets, n: int, docs=None, stream: int | None = None) -> None:
        """Device-pointer variant (torch tensors or raw ints)."""
        check(load().xs_bank_build_device(self.handle, _dptr(seqs), seq_bytes, _dptr(offsets),
                                          _dptr(docs) if docs is not None else None, n, stream))

    def save(self, path: str | Path) -> None:
        Path(path).parent.mkdir(parents=True, exist_ok=True)
        check(load().xs_bank_save(self.handle, str(path).encode()))

    def download(self) -> np.ndarray:
        out = np.empty(self.payload_bytes(), dtype=np.uint8)
        check(load().xs_bank_download(self.handle, _ptr(out), out.size))
        return out

    def upload(self, payload: np.ndarray) -> None:
        p = np.ascontiguousarray(payload, dtype=np.uint8)
        check(load().xs_bank_upload(self.handle, _ptr(p), p.size))

    # ------------------------------------------------------------ queries
    def query(self, reads: PackedReads | Iterable, step: int = 1, want_hits: bool = True,
              hit_dtype=np.uint32, out: np.ndarray | None = None):
        """(hits [n, D], num_kmers [n] uint64) for host reads.

        hit_dtype: np.uint32 (xs_query), np.uint8 / np.uint16 (xs_query_hits:
        narrowed on the device), or "auto": the narrowest of the three that
        holds the largest per-read k-mer count of the batch, which bounds every
        count.  out: a reusable C-contiguous [n, D] array of that dtype (for
        instance from ``pinned_empty``), filled by DMA without page faults."""
        dev = _device_batch(reads)
        if dev:
            reads.check_valid()
        pr = reads if dev or isinstance(reads, PackedReads) else pack_sequences(reads)
        if step < 1:
            raise ValueError("step must be >= 1")
        cols = self.num_docs
        if isinstance(hit_dtype, str) and hit_dtype == "auto":
            hit_dtype = narrowest_count_dtype(_kmers_of(reads.max_len, self.term_size, step) if dev
                                              else max_kmers(pr, self.term_size, step))
        hit_dtype = np.dtype(hit_dtype)
        if hit_dtype not in (np.uint8, np.uint16, np.uint32):
            raise ValueError("hit_dtype must be uint8, uint16 or uint32")
        hits = None
        if want_hits:
            if out is not None:
                if out.shape != (pr.n, cols) or out.dtype != hit_dtype or not out.flags.c_contiguous:
                    raise ValueError(f"out must be a C-contiguous {(pr.n, cols)} {hit_dtype} array")
                hits = out
            else:
                hits = _HOST_POOL.empty((pr.n, cols), hit_dtype)  # recycled pages, see _HostPool
        nk = np.empty(pr.n, dtype=np.uint64)
        if dev:
            check(load().xs_query_hits_device(self.handle, pr.seqs_ptr, pr.seq_bytes, pr.offsets_ptr, pr.n,
                                              pr.max_len, step, _ptr(hits) if hits is not None else None,
                                              hit_dtype.itemsize, _ptr(nk), None))
        else:
            check(load().xs_query_hits(self.handle, _ptr(pr.buf), _ptr(pr.offsets), pr.n, step,
                                       _ptr(hits) if hits is not None else None, hit_dtype.itemsize, _ptr(nk)))
        return hits, nk

    def query_totals(self, reads: PackedReads | Iterable, step: int = 1):
        """(totals [D] uint64, total k-mers) without materialising the hit matrix."""
        if _device_batch(reads):
            reads.check_valid()
            if step < 1:
                raise ValueError("step must be >= 1")
            t = np.zeros(self.num_docs + 1, dtype=np.uint64)
            check(load().xs_query_hits_device(self.handle, reads.seqs_ptr, reads.seq_bytes, reads.offsets_ptr,
                                              reads.n, reads.max_len, step, None, 4, None, _ptr(t)))
            return t[:-1].copy(), int(t[-1])
        pr = reads if isinstance(reads, PackedReads) else pack_sequences(reads)
        tot = np.zeros(self.num_docs, dtype=np.uint64)
        nk = ctypes.c_uint64(0)
        check(load().xs_query_totals(self.handle, _ptr(pr.buf), _ptr(pr.offsets), pr.n, step,
                                     _ptr(tot), ctypes.byref(nk)))
        return tot, int(nk.value)

    def query_best(self, reads: PackedReads | Iterable, step: int = 1, want_totals: bool = False):
        """Per-read best doc (XS_BEST_AMBIGUOUS on ties), its hit count, num_kmers,
        and optionally the D+1 totals; the hit matrix stays on the device."""
        pr = reads if isinstance(reads, PackedReads) else pack_sequences(reads)
        if step < 1:
            raise ValueError("step must be >= 1")
        best = np.empty(pr.n, dtype=np.uint32)
        bh = np.empty(pr.n, dtype=np.uint32)
        nk = np.empty(pr.n, dtype=np.uint64)
        tot = np.empty(self.num_docs + 1, dtype=np.uint64) if want_totals else None
        check(load().xs_query_best(self.handle, _ptr(pr.buf), _ptr(pr.offsets), pr.n, step, _ptr(best),
                                   _ptr(bh), _ptr(nk), _ptr(tot) if tot is not None else None))
        return best, bh, nk, tot

    def query_device(self, seqs, seq_bytes: int, offsets, n: int, step: int = 1, hits=None,
                     num_kmers=None, totals=None, stream: int | None = None) -> None:
        """Enqueue a query on device buffers (torch tensors or raw device pointers)."""
        check(load().xs_query_device(self.handle, _dptr(seqs), seq_bytes, _dptr(offsets), n, step,
                                     _dptr(hits), _dptr(num_kmers), _dptr(totals), stream))

    def mlst_sum(self, chunk_hits: np.ndarray, seq_of_chunk: np.ndarray, n_seqs: int,
                 threshold: int) -> np.ndarray:
        h = np.ascontiguousarray(chunk_hits, dtype=np.uint32)
        s = np.ascontiguousarray(seq_of_chunk, dtype=np.uint32)
        out = np.zeros((n_seqs, self.num_docs), dtype=np.uint64)
        check(load().xs_mlst_sum(self.handle, _ptr(h), _ptr(s), s.size, n_seqs, threshold, _ptr(out)))
        return out

    def mlst_query(self, direct: PackedReads | Iterable, chunks: Iterable, chunk_owner, n_owners: int,
                   step: int = 1, threshold: int = 50):
        """One MLST locus in one call (xs_mlst_query): hit rows of the `direct`
        sequences [n_direct, D] uint32, and for the chunks of the long
        sequences, per owner: summed scores > threshold [n_owners, D] uint64,
        first passing chunk [n_owners, D] uint32 (0xFFFFFFFF: none) and its
        score [n_owners, D] uint32."""
        if step < 1:
            raise ValueError("step must be >= 1")
        dp = direct if isinstance(direct, PackedReads) else pack_sequences(direct)
        cp = pack_sequences(chunks)
        owner = np.ascontiguousarray(chunk_owner, dtype=np.uint32)
        if owner.size != cp.n:
            raise ValueError("one owner per chunk")
        if cp.n:
            buf = np.concatenate([dp.buf[:dp.nbytes], cp.buf])
            offs = np.concatenate([dp.offsets, cp.offsets[1:] + np.uint64(dp.nbytes)])
        else:
            buf, offs = dp.buf, dp.offsets
        D = self.num_docs
        hits = np.empty((dp.n, D), dtype=np.uint32)
        scores = np.empty((n_owners, D), dtype=np.uint64)
        first = np.empty((n_owners, D), dtype=np.uint32)
        fscore = np.empty((n_owners, D), dtype=np.uint32)
        check(load().xs_mlst_query(self.handle, _ptr(buf), _ptr(offs), dp.n, cp.n, _ptr(owner), n_owners, step,
                                   threshold, _ptr(hits) or None, _ptr(scores) or None, _ptr(first) or None,
                                   _ptr(fscore) or None))
        return hits, scores, first, fscore

    def set_profiling(self, on: bool = True) -> None:
        check(load().xs_bank_set_profiling(self.handle, 1 if on else 0))

    def last_probe_ms(self) -> float:
        ms = ctypes.c_float(0.0)
        check(load().xs_bank_last_probe_ms(self.handle, ctypes.byref(ms)))
        return float(ms.value)

    def probe_stats(self) -> tuple[int, float, float]:
        """(launches, total ms, max ms) of the probe kernel since the last call."""
        n = ctypes.c_uint64(0)
        tot = ctypes.c_double(0.0)
        mx = ctypes.c_float(0.0)
        check(load().xs_bank_probe_stats(self.handle, ctypes.byref(n), ctypes.byref(tot), ctypes.byref(mx)))
        return int(n.value), float(tot.value), float(mx.value)

    PASSES = ("prep", "bucket", "lookup", "resolve")

    def pass_stats(self) -> dict:
        """Partitioned probes, profiling on: {pass: (total ms, instances)} since
        the last call (xs_bank_pass_stats; then resets)."""
        ms = np.zeros(4, dtype=np.float64)
        cnt = np.zeros(4, dtype=np.uint64)
        check(load().xs_bank_pass_stats(self.handle, _ptr(ms), _ptr(cnt)))
        return {name: (float(ms[i]), int(cnt[i])) for i, name in enumerate(self.PASSES)}

    def probe_rows(self) -> int:
        """rbloom: filter words loaded by the probes since the last call (profiling on)."""
        n = ctypes.c_uint64(0)
        check(load().xs_bank_probe_rows(self.handle, ctypes.byref(n)))
        return int(n.value)

    def probe_path(self) -> int:
        """Path of the last query: _lib.XS_PATH_GATHER or _lib.XS_PATH_PARTITIONED."""
        v = ctypes.c_int(0)
        check(load().xs_bank_probe_path(self.handle, ctypes.byref(v)))
        return int(v.value)

    def workspace_bytes(self) -> tuple[int, int]:
        """(held, peak) device bytes of this handle's transient workspace
        (xs_bank_workspace_bytes; the bank image not included)."""
        held, peak = ctypes.c_uint64(0), ctypes.c_uint64(0)
        check(load().xs_bank_workspace_bytes(self.handle, ctypes.byref(held), ctypes.byref(peak)))
        return int(held.value), int(peak.value)

    def probe_options(self) -> dict:
        """This handle's path selection (xs_bank_get_probe_options)."""
        o = _lib.ProbeOptions()
        check(load().xs_bank_get_probe_options(self.handle, ctypes.byref(o)))
        return {name: int(getattr(o, name)) for name, _ in o._fields_}

    def set_probe_options(self, **changes) -> dict:
        """Change this handle's path selection (xs_bank_set_probe_options):
        cobs_part 0-4, bloom_part 0-3, workspace_mib, small_calls 0/1;
        unnamed fields keep their values.  The defaults are the
        production paths; every path gives the same results (the tests run
        them all on one bank).  Returns the previous options."""
        old = self.probe_options()
        unknown = set(changes) - set(old)
        if unknown:
            raise TypeError(f"unknown probe options {sorted(unknown)}")
        o = _lib.ProbeOptions(**{**old, **{k: int(v) for k, v in changes.items()}})
        check(load().xs_bank_set_probe_options(self.handle, ctypes.byref(o)))
        return old

    # ------------------------------------------------------------ lifetime
    def close(self) -> None:
        if self._h is not None:
            load().xs_bank_close(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def best_device(hits, n: int, num_docs: int, best, best_hits=None, stream: int | None = None) -> None:
    """xs_best_device: per-read best doc of a device hit matrix (n x num_docs uint32)."""
    check(load().xs_best_device(_dptr(hits), n, num_docs, _dptr(best), _dptr(best_hits), stream))


def gather_reads_device(seqs, offsets, index, m: int, out_seqs, out_offsets, stream: int | None = None) -> None:
    """xs_gather_reads_device: out read j = read index[j] at out_offsets[j]."""
    check(load().xs_gather_reads_device(_dptr(seqs), _dptr(offsets), _dptr(index), m, _dptr(out_seqs),
                                        _dptr(out_offsets), stream))


def _dptr(x) -> int | None:
    """Device pointer of a torch tensor, or an int pointer, or None."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    ptr = getattr(x, "data_ptr", None)
    if ptr is None:
        raise TypeError(f"expected a device tensor or pointer, got {type(x)!r}")
    if not getattr(x, "is_cuda", False):
        raise ValueError("device queries need tensors on the GPU")
    if not x.is_contiguous():
        raise ValueError("device tensors must be contiguous")
    return ptr()


__all__ = ["Bank", "bloom_parameters", "cobs_signature_size", "KIND_NAMES", "pinned_empty", "max_kmers",
           "XS_BANK_COBS_CLASSIC", "XS_BANK_COBS_COMPACT", "XS_BANK_RBLOOM", "_lib"]
