"""FASTA/FASTQ input of the probe path, parsed natively.

Mirrors what the hot path consumes from ``src/xspect/file_io.py:47-79``
(``get_record_iterator``: Bio.SeqIO parse by file extension).  Files are read
by the multithreaded reader in libxspect_hip.so (``xs_fastx_*``), which yields
batches already packed for the probe call; ``get_record_iterator`` builds
``Record`` objects (``.id`` = first header token, ``.seq``) from them for
callers that want records.  Bio.SeqRecord objects are accepted anywhere a
record is expected.
"""
from __future__ import annotations

import os

import ctypes
import functools
from dataclasses import dataclass
from pathlib import Path
from typing import Iterator

import numpy as np

from ._lib import (XS_ERR_FORMAT, XS_FASTX_FASTA, XS_FASTX_FASTQ, XS_FASTX_PINNED, FastxBatch, FastxDBatch,
                   check, load)
from .packing import PackedIds, PackedReads

FASTA_ENDINGS = ["fasta", "fna", "fa", "ffn", "frn"]  # definitions.py:6
FASTQ_ENDINGS = ["fastq", "fq"]                       # definitions.py:7
# File text per native reader batch.
DEFAULT_BATCH_TEXT = 256 << 20


def file_reader_device(index) -> int | None:
    """The device a model's file inputs are read on (the reader's device mode,
    text straight to HBM, records found there), or None for the host reader:
    device mode when the index is a GPU bank (bank.Bank), unless
    XSPECT2_AMD_READER=host (an operational setting, read once per process)."""
    from .bank import Bank

    if _host_reader_forced():
        return None
    return index.device if isinstance(index, Bank) else None


@functools.lru_cache(maxsize=None)
def _host_reader_forced() -> bool:
    return os.environ.get("XSPECT2_AMD_READER", "device").strip().lower() == "host"


@dataclass
class Record:
    id: str
    seq: str
    description: str = ""

    def __len__(self) -> int:
        return len(self.seq)


def is_record(obj) -> bool:
    return hasattr(obj, "id") and hasattr(obj, "seq")


def seq_text(obj) -> str:
    """The sequence text of a str / bytes / Bio.Seq."""
    if isinstance(obj, str):
        return obj
    if isinstance(obj, (bytes, bytearray)):
        return bytes(obj).decode("ascii")
    return str(obj)


class SeqBatch:
    """One batch of the native reader: packed sequences (zero-copy views of
    the reader's buffers, valid until the reader's second following call)
    and the record ids."""

    def __init__(self, fb):
        n = int(fb.n)
        self.n = n
        self.text_offset = int(fb.text_offset)
        self.text_bytes = int(fb.text_bytes)
        if n:
            offs = np.ctypeslib.as_array(ctypes.cast(fb.offsets, ctypes.POINTER(ctypes.c_uint64)), (n + 1,))
            # +1: the reader keeps 64 defined bytes past the end (the guard byte
            # PackedReads carries)
            buf = np.ctypeslib.as_array(ctypes.cast(fb.seqs, ctypes.POINTER(ctypes.c_uint8)),
                                        (int(fb.seq_bytes) + 1,))
            ioffs = np.ctypeslib.as_array(ctypes.cast(fb.id_offsets, ctypes.POINTER(ctypes.c_uint64)), (n + 1,))
            self._ids_raw = ctypes.string_at(fb.ids, int(ioffs[n])) if ioffs[n] else b""
            self._ioffs = ioffs.copy()
            doffs = np.ctypeslib.as_array(ctypes.cast(fb.desc_offsets, ctypes.POINTER(ctypes.c_uint64)), (n + 1,))
            self._descs_raw = ctypes.string_at(fb.descs, int(doffs[n])) if doffs[n] else b""
            self._doffs = doffs.copy()
        else:
            offs = np.zeros(1, dtype=np.uint64)
            buf = np.zeros(1, dtype=np.uint8)
            self._ids_raw, self._ioffs = b"", np.zeros(1, dtype=np.uint64)
            self._descs_raw, self._doffs = b"", np.zeros(1, dtype=np.uint64)
        self.packed = PackedReads(buf, offs)

    def ids(self) -> list[str]:
        raw, o = self._ids_raw, self._ioffs.tolist()
        if raw.isascii():
            s = raw.decode("ascii")
            return [s[o[i]:o[i + 1]] for i in range(self.n)]
        return [raw[o[i]:o[i + 1]].decode("utf-8", errors="replace") for i in range(self.n)]

    def ids_packed(self) -> PackedIds:
        """The ids as one buffer + offsets (no Python string per read)."""
        return PackedIds(self._ids_raw, self._ioffs)

    def descriptions(self) -> list[str]:
        """Record titles (header line without '>'/'@', right-stripped)."""
        raw, o = self._descs_raw, self._doffs.tolist()
        return [raw[o[i]:o[i + 1]].decode("utf-8", errors="replace") for i in range(self.n)]

    def lengths(self) -> np.ndarray:
        return self.packed.lengths()

    def write_fasta(self, path: Path, index: np.ndarray | None = None, append: bool = True) -> None:
        """Append records (all, or those in `index`) to a FASTA file the way
        Bio.SeqIO.write(record, fh, "fasta") does (file_io.py:188-191)."""
        idx = None if index is None else np.ascontiguousarray(index, dtype=np.uint32)
        n = self.n if idx is None else int(idx.size)
        vp = ctypes.c_void_p
        check(load().xs_write_fasta(str(path).encode(), 1 if append else 0, vp(self.packed.buf.ctypes.data),
                                    vp(self.packed.offsets.ctypes.data), self._descs_raw,
                                    vp(self._doffs.ctypes.data), vp(idx.ctypes.data) if idx is not None and n else None,
                                    n, 60))

    def records(self) -> list[Record]:
        buf, o = self.packed.buf, self.packed.offsets.tolist()
        raw = buf[:o[-1]].tobytes() if self.n else b""
        return [Record(rid, raw[o[i]:o[i + 1]].decode("ascii", errors="replace"))
                for i, rid in enumerate(self.ids())]


class DeviceSeqBatch:
    """One batch of the reader's device mode (xs_fastx_next_device): the
    packed sequences and their offsets are in HBM (``seqs_ptr``,
    ``offsets_ptr``), ids, titles and a copy of the offsets in the reader's
    pinned host buffers, copied out on first use.  All of them are valid until
    the reader's second following batch: ``check_valid`` (run by every access
    and by ``Bank.query`` / ``query_totals``, which take the batch as they take
    a PackedReads) raises for a batch whose reader was closed or has moved two
    batches on, whose memory is freed or reused."""

    def __init__(self, fb: FastxDBatch, reader: "FastxReader"):
        self._reader = reader
        self._gen = reader._gen
        self.n = int(fb.n)
        self.seq_bytes = int(fb.seq_bytes)
        self.seqs_ptr = int(fb.seqs or 0)
        self.offsets_ptr = int(fb.offsets or 0)
        self.max_len = int(fb.max_len)
        self.parsed_on_device = bool(fb.parsed_on_device)
        self.text_offset = int(fb.text_offset)
        self.text_bytes = int(fb.text_bytes)
        self._host = (fb.host_offsets, fb.ids, fb.id_offsets, fb.descs, fb.desc_offsets)
        self._fb = fb  # host_ready: the host arrays land behind the caller's probe of the batch
        self._host_waited = not fb.host_ready
        self._offsets = self._ids_raw = self._descs_raw = None

    def check_valid(self) -> None:
        rd = self._reader
        if rd._h is None or rd._gen - self._gen > 1:
            raise RuntimeError("device batch is no longer valid: its reader was closed or has read two batches "
                               "since (the device buffers are freed or reused)")

    def _wait_host(self) -> None:
        """Block until the batch's host arrays (offsets, ids, titles) have landed."""
        if not self._host_waited:
            check(load().xs_fastx_wait_host(ctypes.byref(self._fb)))
            self._host_waited = True

    def _u64(self, ptr) -> np.ndarray:
        self._wait_host()
        return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint64)), (self.n + 1,)).copy()

    @property
    def offsets(self) -> np.ndarray:
        if self._offsets is None:
            self.check_valid()
            self._offsets = self._u64(self._host[0]) if self.n else np.zeros(1, dtype=np.uint64)
        return self._offsets

    def _text(self, which: int):
        self.check_valid()
        if not self.n:
            return b"", np.zeros(1, dtype=np.uint64)
        self._wait_host()
        o = self._u64(self._host[which + 1])
        return (ctypes.string_at(self._host[which], int(o[-1])) if o[-1] else b""), o

    def ids(self) -> list[str]:
        if self._ids_raw is None:
            self._ids_raw, self._ioffs = self._text(1)
        return SeqBatch.ids(self)

    def ids_packed(self) -> PackedIds:
        if self._ids_raw is None:
            self._ids_raw, self._ioffs = self._text(1)
        return PackedIds(self._ids_raw, self._ioffs)

    def descriptions(self) -> list[str]:
        if self._descs_raw is None:
            self._descs_raw, self._doffs = self._text(3)
        return SeqBatch.descriptions(self)

    def lengths(self) -> np.ndarray:
        return np.diff(self.offsets)

    def to_host(self) -> PackedReads:
        """The sequences copied back from HBM (tests, diagnostics)."""
        self.check_valid()
        buf = np.zeros(self.seq_bytes + 1, dtype=np.uint8)
        if self.seq_bytes:
            check(load().xs_memcpy_to_host(buf.ctypes.data, self.seqs_ptr, self.seq_bytes))
        return PackedReads(buf, self.offsets.copy())


def fastx_format(path: Path) -> int:
    """XS_FASTX_* of a path by its ending (file_io.py:72-79), else ValueError."""
    ending = Path(path).suffix[1:]
    if ending in FASTA_ENDINGS:
        return XS_FASTX_FASTA
    if ending in FASTQ_ENDINGS:
        return XS_FASTX_FASTQ
    raise ValueError("Invalid file format, must be a fasta or fastq file")


class FastxReader:
    """Native multithreaded FASTA/FASTQ reader (xs_fastx_* in xspect_hip.h).

    ``part``/``parts``: read only part ``part`` of ``parts`` byte ranges of the
    file, cut at record starts (xs_fastx_open_range): one rank's share of a
    read-sharded job.  The parts' records in part order are the file's.

    ``device``: a HIP device ordinal selects the device mode
    (xs_fastx_open_device): each window's text goes to HBM and its records are
    found on the GPU; batches are DeviceSeqBatch."""

    def __init__(self, path: Path, threads: int = 0, pinned: bool = False, part: int = 0, parts: int = 1,
                 device: int | None = None):
        self.path = Path(path)
        fmt = fastx_format(self.path)
        if not 0 <= part < parts:
            raise ValueError("part must be in [0, parts)")
        self._lib = load()
        self._h = None
        self._gen = 0  # batches read (device batches check their age against it)
        self.device = device
        h = ctypes.c_void_p()
        if device is not None:
            check(self._lib.xs_fastx_open_device(str(self.path).encode(), fmt, threads, device, part, parts,
                                                 ctypes.byref(h)))
        else:
            check(self._lib.xs_fastx_open_range(str(self.path).encode(), fmt, threads,
                                                XS_FASTX_PINNED if pinned else 0, part, parts, ctypes.byref(h)))
        self._h = h

    def next_batch(self, max_bytes: int = DEFAULT_BATCH_TEXT) -> SeqBatch:
        """Next batch (n == 0 at end of file).  Malformed records raise ValueError."""
        if self._h is None:
            raise ValueError("reader is closed")
        self._gen += 1
        if self.device is not None:
            fb = FastxDBatch()
            rc = self._lib.xs_fastx_next_device(self._h, max_bytes, ctypes.byref(fb))
        else:
            fb = FastxBatch()
            rc = self._lib.xs_fastx_next(self._h, max_bytes, ctypes.byref(fb))
        if rc == XS_ERR_FORMAT:
            raise ValueError(self._lib.xs_last_error().decode())
        check(rc)
        return DeviceSeqBatch(fb, self) if self.device is not None else SeqBatch(fb)

    def batches(self, max_bytes: int = DEFAULT_BATCH_TEXT) -> Iterator[SeqBatch]:
        while True:
            b = self.next_batch(max_bytes)
            if b.n == 0:
                return
            yield b

    def close(self) -> None:
        if self._h:
            self._lib.xs_fastx_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_batches(path: Path, max_bytes: int | None = None, threads: int = 0,
                 pinned: bool = False, part: int = 0, parts: int = 1,
                 device: int | None = None) -> Iterator[SeqBatch]:
    """Batches of a FASTA/FASTQ file (or of its part ``part`` of ``parts``),
    parsing batch i+1 while the caller works on batch i (the native reader
    releases the GIL).  A yielded batch's buffers stay valid until the
    generator is advanced again.  max_bytes: file text per batch (None:
    DEFAULT_BATCH_TEXT).  device: read in device mode on that GPU
    (DeviceSeqBatch); then the next window's text loads while the caller
    works, and its records are found on the GPU when the caller asks for it."""
    from concurrent.futures import ThreadPoolExecutor

    max_bytes = DEFAULT_BATCH_TEXT if max_bytes is None else max_bytes

    if device is not None:
        # device mode: the next window's text already loads behind the
        # caller's work (the reader's own prefetch thread); parsing it on the
        # GPU beside the caller's probe only slows both, so the parse waits
        # for the caller (file -> totals of 1 M reads: 16.4 ms this way,
        # 17.6 ms with the parse on a worker thread,
        # profiles/r04_e2e_parse_overlap.txt)
        with FastxReader(path, threads, pinned, part, parts, device) as rd:
            while True:
                b = rd.next_batch(max_bytes)
                if b.n == 0:
                    return
                yield b

    with FastxReader(path, threads, pinned, part, parts, device) as rd, ThreadPoolExecutor(1) as pool:
        fut = pool.submit(rd.next_batch, max_bytes)
        while True:
            b = fut.result()
            if b.n == 0:
                return
            # the reader double-buffers: parsing i+1 leaves batch i intact
            fut = pool.submit(rd.next_batch, max_bytes)
            yield b


@dataclass(frozen=True)
class FileShard:
    """Part ``part`` of ``parts`` of a FASTA/FASTQ file (record-aligned byte
    ranges): what one rank of a read-sharded job classifies.  Accepted by the
    models' ``predict_columnar`` / ``predict_matrix`` like a Path."""
    path: Path
    part: int = 0
    parts: int = 1

    def batches(self, max_bytes: int | None = None) -> Iterator[SeqBatch]:
        return read_batches(self.path, max_bytes, part=self.part, parts=self.parts)


def _native_records(path: Path) -> Iterator[Record]:
    for b in read_batches(path):
        yield from b.records()


def get_record_iterator(file_path: Path) -> Iterator[Record]:
    """Record iterator of a FASTA/FASTQ file (error messages as file_io.py:66-79)."""
    check_input_path(file_path)
    return _native_records(file_path)


def check_input_path(file_path) -> int:
    """The input checks of get_record_iterator (file_io.py:66-79); XS_FASTX_* format."""
    if not isinstance(file_path, Path):
        raise ValueError("Path must be a Path object")
    if not file_path.exists():
        raise ValueError("File does not exist")
    if not file_path.is_file():
        raise ValueError("Path must be a file")
    return fastx_format(file_path)


def write_fasta(records, path: Path, width: int = 0) -> None:
    path = Path(path)
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", encoding="utf-8") as fh:
        for r in records:
            s = seq_text(r.seq)
            fh.write(f">{r.id}\n")
            if width:
                for i in range(0, len(s), width):
                    fh.write(s[i:i + width] + "\n")
            else:
                fh.write(s + "\n")


def prepare_input_output_paths(input_path: Path):
    """Input files + output-path factory (mirror of file_io.py:194-234).

    A directory yields its files grouped by ending in the order of
    FASTA_ENDINGS + FASTQ_ENDINGS, each group in ``glob`` (directory) order
    as the reference's (file_io.py:218-221), and suffixes every output name
    with _<idx+1>, so output file i belongs to the same input as there.
    """
    input_path = Path(input_path)
    input_is_dir = input_path.is_dir()
    if input_is_dir:
        inputs = [p for e in FASTA_ENDINGS + FASTQ_ENDINGS for p in input_path.glob(f"*.{e}")]
    elif input_path.is_file():
        inputs = [input_path]
    else:
        raise ValueError("Invalid input path")

    def get_output_path(idx: int, output_path: Path) -> Path:
        output_path = Path(output_path)
        if input_is_dir:
            return output_path.parent / f"{output_path.stem}_{idx + 1}{output_path.suffix}"
        return output_path

    return inputs, get_output_path


def filter_sequences(input_file: Path, output_file: Path, included_ids: list[str]) -> None:
    """Where the reference keeps it (file_io.py:166-191): the records of
    `input_file` whose ids are in `included_ids`, written as FASTA; the
    implementation is xspect2_amd.filter_sequences.filter_sequences."""
    from .filter_sequences import filter_sequences as _filter
    return _filter(input_file, output_file, included_ids)
