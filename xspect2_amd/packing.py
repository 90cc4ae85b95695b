"""Batch packing of reads for one C-ABI call.

The reference hands COBS one ``str(sequence)`` per read
(``probabilistic_filter_model.py:227``); here every read of a batch is
concatenated into one byte buffer with ``n+1`` uint64 offsets.
"""
from __future__ import annotations

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
