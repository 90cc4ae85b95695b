"""Batch packing of reads for one C-ABI call.

The reference hands COBS one ``str(sequence)`` per read
(``probabilistic_filter_model.py:227``); here every read of a batch is
concatenated into one byte buffer with ``n+1`` uint64 offsets.
"""
from __future__ import annotations

from collections.abc import Sequence
from dataclasses import dataclass
from typing import Iterable

import numpy as np


@dataclass
class PackedReads:
    buf: np.ndarray       # uint8, concatenated sequence bytes (+1 guard byte)
    offsets: np.ndarray   # uint64 [n+1]

    @property
    def n(self) -> int:
        return int(self.offsets.size - 1)

    @property
    def nbytes(self) -> int:
        return int(self.offsets[-1]) if self.offsets.size else 0

    def lengths(self) -> np.ndarray:
        return np.diff(self.offsets)


def _as_bytes(s) -> bytes:
    if isinstance(s, bytes):
        return s
    if isinstance(s, str):
        return s.encode("ascii", errors="strict")
    if isinstance(s, (bytearray, memoryview)):
        return bytes(s)
    return str(s).encode("ascii", errors="strict")


def pack_sequences(seqs: Iterable) -> PackedReads:
    """Concatenate str/bytes/Seq-like sequences."""
    parts = [_as_bytes(s) for s in seqs]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    if parts:
        np.cumsum(np.fromiter((len(p) for p in parts), dtype=np.uint64, count=len(parts)), out=offs[1:])
    buf = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8)
    return PackedReads(buf, offs)


def pack_fixed(arr: np.ndarray) -> PackedReads:
    """Pack an [n, L] uint8 matrix of equal-length reads without copying rows."""
    a = np.ascontiguousarray(arr, dtype=np.uint8)
    n, L = a.shape
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
    buf = np.concatenate([a.reshape(-1), np.zeros(1, dtype=np.uint8)])
    return PackedReads(buf, offs)


class PackedIds(Sequence):
    """Read ids as the native reader hands them over: one byte buffer and n+1
    offsets.  A result of millions of reads keeps its ids so (MatrixResult):
    Python strings are made only when a caller reads them, decoded as
    ``SeqBatch.ids`` decodes them (ASCII, else UTF-8 with replacement), and
    ``MatrixResult.save`` quotes them natively (xs_ids_json_quote).  Equal to
    a list of the same strings."""

    __slots__ = ("buf", "offs", "_list", "_ascii")

    def __init__(self, buf: bytes, offs):
        self.offs = np.ascontiguousarray(offs, dtype=np.uint64)
        lo, hi = (int(self.offs[0]), int(self.offs[-1])) if self.offs.size else (0, 0)
        self.buf = bytes(buf[lo:hi]) if lo else bytes(buf[:hi])
        if lo:
            self.offs = self.offs - np.uint64(lo)
        self._list = None
        self._ascii = None

    @classmethod
    def concat(cls, parts) -> "PackedIds":
        parts = list(parts)
        if len(parts) == 1:
            return parts[0]
        offs = [np.zeros(1, dtype=np.uint64)]
        base = 0
        for p in parts:
            offs.append(p.offs[1:] + np.uint64(base))
            base += len(p.buf)
        return cls(b"".join(p.buf for p in parts), np.concatenate(offs))

    @classmethod
    def of(cls, ids) -> "PackedIds":
        """From strings (UTF-8)."""
        enc = [s.encode("utf-8") for s in ids]
        offs = np.zeros(len(enc) + 1, dtype=np.uint64)
        if enc:
            np.cumsum(np.fromiter(map(len, enc), dtype=np.uint64, count=len(enc)), out=offs[1:])
        return cls(b"".join(enc), offs)

    def __len__(self) -> int:
        return int(self.offs.size - 1)

    @property
    def is_ascii(self) -> bool:
        if self._ascii is None:
            self._ascii = self.buf.isascii()
        return self._ascii

    def tolist(self) -> list[str]:
        if self._list is None:
            o = self.offs.tolist()
            n = len(self)
            if self.is_ascii:
                s = self.buf.decode("ascii")
                self._list = [s[o[i]:o[i + 1]] for i in range(n)]
            else:
                b = self.buf
                self._list = [b[o[i]:o[i + 1]].decode("utf-8", errors="replace") for i in range(n)]
        return self._list

    def __getitem__(self, i):
        if isinstance(i, slice):
            a, b, st = i.indices(len(self))
            if st != 1:
                return self.tolist()[i]
            b = max(a, b)
            return PackedIds(self.buf, self.offs[a:b + 1])
        return self.tolist()[i]

    def __iter__(self):
        return iter(self.tolist())

    def index(self, s: str) -> int:
        """Position of the first id equal to `s` (ValueError if none), found by
        a byte search of the buffer for ASCII ids: no Python string per id."""
        if not isinstance(s, str) or not (self.is_ascii and s.isascii()) or self._list is not None or not s:
            return self.tolist().index(s)
        key = s.encode("ascii")
        starts = self.offs[:-1]
        pos = self.buf.find(key)
        while pos >= 0:
            lo, hi = np.searchsorted(starts, pos, side="left"), np.searchsorted(starts, pos, side="right")
            for i in range(int(lo), int(hi)):
                if int(self.offs[i + 1]) == pos + len(key):
                    return i
            pos = self.buf.find(key, pos + 1)
        raise ValueError(f"{s!r} is not in the ids")

    def __contains__(self, s) -> bool:
        if not isinstance(s, str):
            return False
        if not (self.is_ascii and s.isascii()) or self._list is not None:
            return s in self.tolist()
        key = s.encode("ascii")
        if not key:
            return bool(np.any(self.offs[1:] == self.offs[:-1]))
        starts = self.offs[:-1]
        pos = self.buf.find(key)
        while pos >= 0:
            # ids starting at pos (empty ids share their start with the next one)
            lo, hi = np.searchsorted(starts, [pos, pos], side="left")[0], np.searchsorted(starts, pos, side="right")
            for i in range(int(lo), int(hi)):
                if int(self.offs[i + 1]) == pos + len(key):
                    return True
            pos = self.buf.find(key, pos + 1)
        return False

    def __eq__(self, other) -> bool:
        if isinstance(other, PackedIds):
            return self.buf == other.buf and np.array_equal(self.offs, other.offs) or self.tolist() == other.tolist()
        if isinstance(other, (list, tuple)):
            return self.tolist() == list(other)
        return NotImplemented

    def __repr__(self) -> str:
        return f"PackedIds(n={len(self)}, bytes={len(self.buf)})"

    def has_duplicates(self) -> bool:
        """Whether two ids are equal (native hash for ASCII ids)."""
        if not self.is_ascii:
            return len(set(self.tolist())) != len(self)
        import ctypes

        from ._lib import check, load
        flag = ctypes.c_int(0)
        check(load().xs_ids_has_duplicates(self.buf, ctypes.c_void_p(self.offs.ctypes.data), len(self),
                                           ctypes.byref(flag)))
        return bool(flag.value)

    def drop(self, index) -> "PackedIds":
        """All ids but those at `index` (int array), in order, still packed:
        one pass over the bytes that stay (a few dropped ids of a large shard
        cost what they are, not a gather of every kept byte)."""
        idx = np.unique(np.asarray(index, dtype=np.int64))
        n = len(self)
        lens = (self.offs[1:] - self.offs[:-1]).astype(np.int64)
        starts = self.offs[:-1][idx].astype(np.int64)
        dl = lens[idx]
        cut = np.zeros(dl.size + 1, dtype=np.int64)
        np.cumsum(dl, out=cut[1:])
        gone = np.repeat(starts - cut[:-1], dl) + np.arange(int(cut[-1]), dtype=np.int64)
        buf = np.delete(np.frombuffer(self.buf, dtype=np.uint8), gone).tobytes()
        keep = np.ones(n, dtype=bool)
        keep[idx] = False
        offs = np.zeros(n - idx.size + 1, dtype=np.uint64)
        np.cumsum(lens[keep], out=offs[1:])
        return PackedIds(buf, offs)

    def take(self, index) -> "PackedIds":
        """The ids at `index` (int array), in that order, still packed."""
        idx = np.asarray(index, dtype=np.int64)
        starts = self.offs[:-1][idx].astype(np.int64)
        lens = self.offs[1:][idx].astype(np.int64) - starts
        offs = np.zeros(idx.size + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        pos = np.repeat(starts - offs[:-1].astype(np.int64), lens) + np.arange(int(offs[-1]), dtype=np.int64)
        return PackedIds(np.frombuffer(self.buf, dtype=np.uint8)[pos].tobytes(), offs)

    def hash128(self) -> np.ndarray:
        """[n, 2] uint64: XXH64 of every id's bytes with two seeds (xs_ids_hash128)."""
        import ctypes

        from ._lib import check, load
        out = np.zeros((len(self), 2), dtype=np.uint64)
        if len(self):
            check(load().xs_ids_hash128(self.buf, ctypes.c_void_p(self.offs.ctypes.data), len(self),
                                        ctypes.c_void_p(out.ctypes.data)))
        return out

    def json_packed(self) -> tuple[bytes, np.ndarray]:
        """json.dumps(id) of every id, packed, and n+1 offsets."""
        n = len(self)
        if not self.is_ascii:
            import json
            enc = [json.dumps(s).encode("ascii") for s in self.tolist()]
            off = np.zeros(n + 1, dtype=np.uint64)
            if enc:
                np.cumsum(np.fromiter(map(len, enc), dtype=np.uint64, count=n), out=off[1:])
            return b"".join(enc), off
        import ctypes

        from ._lib import check, load
        cap = 6 * len(self.buf) + 2 * n + 1
        out = ctypes.create_string_buffer(cap)
        off = np.zeros(n + 1, dtype=np.uint64)
        check(load().xs_ids_json_quote(self.buf, ctypes.c_void_p(self.offs.ctypes.data), n,
                                       ctypes.cast(out, ctypes.c_void_p), cap, ctypes.c_void_p(off.ctypes.data)))
        return out.raw[:int(off[-1])], off
