"""Species model over a COBS classic bank resident in HBM.

Drop-in for ``xspect.models.probabilistic_filter_model.ProbabilisticFilterModel``
(reference ``src/xspect/models/probabilistic_filter_model.py:28-601``): same
constructor, ``fit``/``save``/``load``/``predict``/``calculate_hits``/
``to_dict``/``slug`` and the same ``ModelResult``.  What changes is below the
surface: the reference re-enters ``cobs_index.Search.search`` once per read
(``:291-310``, ``:227``); here a whole batch of reads is one call into
libxspect_hip.so, which probes the bank on the GPU.
"""
from __future__ import annotations

import json
import math
from pathlib import Path
from typing import Iterable

import numpy as np

from .bank import Bank, cobs_signature_size
from ._lib import XS_BANK_COBS_CLASSIC
from .file_io import (FASTA_ENDINGS, FASTQ_ENDINGS, FileShard, check_input_path, file_reader_device,
                      get_record_iterator, is_record, read_batches, seq_text)
from .packing import PackedIds, PackedReads, pack_sequences
from .result import MatrixResult, ModelResult
from .util import default_device, slugify

# One C-ABI call handles at most this many sequence bytes / reads.
MAX_BATCH_BYTES = 1 << 30
MAX_BATCH_READS = 1 << 24


def training_files(dir_path: Path) -> list[Path]:
    """Training FASTA/FASTQ files of a species directory in ``iterdir()`` order
    (reference probabilistic_filter_model.py:170-171)."""
    return [f for f in dir_path.iterdir() if f.is_file() and f.suffix[1:] in FASTA_ENDINGS + FASTQ_ENDINGS]


def _records(sequence_input) -> list | None:
    """Materialise a record list / iterator; None if the input is neither."""
    if isinstance(sequence_input, (list, tuple)):
        return list(sequence_input) if all(is_record(r) for r in sequence_input) else None
    if isinstance(sequence_input, (str, bytes, Path)) or is_record(sequence_input):
        return None
    if hasattr(sequence_input, "__iter__") and hasattr(sequence_input, "__next__"):
        return list(sequence_input)
    return None


def _check_seq_type(sequence) -> str:
    """The reference accepts only Bio.Seq here (:219-222); str/bytes are the
    offline stand-ins.  Records and other objects are rejected."""
    if is_record(sequence) or not isinstance(sequence, (str, bytes, bytearray)) and \
            type(sequence).__name__ not in ("Seq", "MutableSeq"):
        raise ValueError("Invalid sequence, must be a Bio.Seq or a Bio.SeqRecord object")
    return seq_text(sequence)


def cobs_result_order(row: np.ndarray) -> np.ndarray:
    """Doc order of one COBS result: score descending, ties by doc index
    (the tie order of the real library is implementation-defined)."""
    return np.argsort(-row.astype(np.int64), kind="stable")


class ProbabilisticFilterModel:
    """Probabilistic filter (COBS classic) species model on the GPU."""

    def __init__(
        self,
        k: int,
        model_display_name: str,
        author: str | None,
        author_email: str | None,
        model_type: str,
        base_path: Path,
        fpr: float = 0.01,
        num_hashes: int = 7,
        training_accessions: dict[str, list[str]] | None = None,
    ) -> None:
        if k < 1:
            raise ValueError("Invalid k value, must be greater than 0")
        if not model_display_name:
            raise ValueError("Invalid filter display name, must be a non-empty string")
        if not model_type:
            raise ValueError("Invalid filter type, must be a non-empty string")
        if not isinstance(base_path, Path):
            raise ValueError("Invalid base path, must be a pathlib.Path object")
        self.k = k
        self.model_display_name = model_display_name
        self.author = author
        self.author_email = author_email
        self.model_type = model_type
        self.base_path = base_path
        self.display_names: dict[str, str] = {}
        self.fpr = fpr
        self.num_hashes = num_hashes
        self.index: Bank | None = None
        self.training_accessions = training_accessions
        self.device = default_device()

    # ------------------------------------------------------------ identity
    def get_cobs_index_path(self) -> str:
        return str(self.base_path / self.slug() / "index.cobs_classic")

    def to_dict(self) -> dict:
        return {
            "model_slug": self.slug(),
            "k": self.k,
            "model_display_name": self.model_display_name,
            "author": self.author,
            "author_email": self.author_email,
            "model_type": self.model_type,
            "model_class": self.__class__.__name__,
            "display_names": self.display_names,
            "fpr": self.fpr,
            "num_hashes": self.num_hashes,
            "training_accessions": self.training_accessions,
        }

    def slug(self) -> str:
        return slugify(self.model_display_name + "-" + str(self.model_type))

    # ------------------------------------------------------------ training
    def fit(self, dir_path: Path, display_names: dict | None = None,
            training_accessions: dict[str, list[str]] | None = None) -> None:
        """Build the COBS classic bank from one FASTA/FASTQ file per species
        (reference :131-194).  Files are taken in ``dir_path.iterdir()`` order,
        as the reference adds them to its DocumentList (:170-179), so
        ``display_names`` keeps the reference's key order (which ``_get_svm``'s
        column indices follow); docs are in the same order (COBS keeping its
        list order is unverified offline).  The doc name is the
        file name up to its first '.' (as COBS does)."""
        display_names = display_names or {}
        if not isinstance(dir_path, Path):
            raise ValueError("Invalid directory path, must be a pathlib.Path object")
        if not dir_path.exists():
            raise ValueError("Directory path does not exist")
        if not dir_path.is_dir():
            raise ValueError("Directory path must be a directory")
        self.training_accessions = training_accessions
        files = training_files(dir_path)
        for f in files:
            if f.stem in display_names:
                self.display_names[f.stem.split(".")[0]] = display_names[f.stem]
            else:
                self.display_names[f.stem.split(".")[0]] = f.stem
        if not files:
            raise ValueError("No valid files found in directory. Must be fasta or fastq")
        names = [f.stem.split(".")[0] for f in files]
        # signature size from the largest document's term count
        terms = [sum(int(np.maximum(b.lengths().astype(np.int64) - self.k + 1, 0).sum())
                     for b in read_batches(f)) for f in files]
        sig = cobs_signature_size(max(max(terms), 1), self.num_hashes, self.fpr)
        bank = Bank.create_cobs(self.k, self.num_hashes, [sig], len(files), names, device=self.device)
        for d, f in enumerate(files):
            for b in read_batches(f):
                bank.build(b.packed, np.full(b.n, d, dtype=np.uint32))
        path = Path(self.get_cobs_index_path())
        bank.save(path)
        if self.index is not None:
            self.index.close()
        self.index = bank

    # ------------------------------------------------------------ queries
    def _query(self, packed, step: int):
        """(hits, num_kmers) of one batch (PackedReads or a device-mode reader
        batch); the hit matrix comes back in the
        narrowest integer type that holds the batch's largest k-mer count."""
        if self.index is None:
            raise ValueError("The model has not been trained yet")
        return self.index.query(packed, step=step, hit_dtype="auto")

    def _hit_dict(self, row: np.ndarray, exclude_ids) -> dict:
        names = self.index.doc_names
        order = cobs_result_order(row)
        vals = row[order].tolist()
        out = {names[i]: v for i, v in zip(order.tolist(), vals)}
        if exclude_ids:
            return {doc: s for doc, s in out.items() if doc not in exclude_ids}
        return out

    def calculate_hits(self, sequence, exclude_ids: list[str] | None = None, step: int = 1) -> dict:
        """{doc_name: score} of one sequence (reference :196-235)."""
        text = _check_seq_type(sequence)
        if not len(text) > self.k:
            raise ValueError("Invalid sequence, must be longer than k")
        hits, _ = self._query(pack_sequences([text]), step)
        return self._hit_dict(hits[0], exclude_ids)

    def predict_matrix(self, sequence_input, step: int = 1):
        """Columnar result of a batch: (ids, hits [n, D], num_kmers [n] uint64);
        hits are uint8 / uint16 / uint32, the narrowest type the reads' k-mer
        counts need.

        Same hits as ``predict`` without per-read dictionaries (the form that
        scales to 10^8 reads)."""
        ids, _, hits, nk = self._matrix(sequence_input, step)
        return ids, hits, nk

    def _matrix(self, sequence_input, step: int):
        if step < 1:
            raise ValueError("step must be >= 1")
        if isinstance(sequence_input, Path):
            return self._matrix_file(sequence_input, step)
        if isinstance(sequence_input, FileShard):
            return self._matrix_file(sequence_input.path, step, sequence_input.part, sequence_input.parts)
        records = self._collect(sequence_input)
        ids = [r.id for r in records]
        texts = [seq_text(r.seq) for r in records]
        lens = [len(t) for t in texts]
        for n in lens:
            if not n > self.k:
                raise ValueError("Invalid sequence, must be longer than k")
        if self.index is None:
            raise ValueError("The model has not been trained yet")
        parts = [self._query(pack_sequences(texts[lo:hi]), step) for lo, hi in _batches(lens)]
        return ids, lens, *_stack(parts, self.index.num_docs)

    def _matrix_file(self, path: Path, step: int, part: int = 0, parts: int = 1):
        """A FASTA/FASTQ file (or its part ``part`` of ``parts``, FileShard)
        streamed through the native reader: batch i+1 is parsed while batch i
        is probed, and no per-record objects are built (the reference iterates
        Bio.SeqIO records, :316-330).  On a GPU bank the reader runs in device
        mode (file_io.file_reader_device): the window's text goes to HBM and
        the probe reads the records there."""
        check_input_path(path)
        if self.index is None:
            raise ValueError("The model has not been trained yet")
        ids: list[PackedIds] = []
        lens, hits, nks = [], [], []
        dev = file_reader_device(self.index)
        for batch in read_batches(path, part=part, parts=parts, device=dev):
            # probe first: a device batch's host arrays (offsets, ids) land
            # behind the probe; a read no longer than k has no k-mers there, and
            # the batch raises below exactly as it would have before the probe
            h, n = self._query(batch if dev is not None else batch.packed, step)
            L = batch.lengths()
            if (L <= self.k).any():
                raise ValueError("Invalid sequence, must be longer than k")
            ids.append(batch.ids_packed())  # the reader's id buffer: no string per read
            lens.append(L)
            hits.append(h)
            nks.append(n)
        hits_m, nk = _stack(list(zip(hits, nks)), self.index.num_docs)
        lens_a = np.concatenate(lens) if lens else np.zeros(0, dtype=np.uint64)
        return PackedIds.concat(ids) if ids else [], lens_a, hits_m, nk

    def _collect(self, sequence_input) -> list:
        if is_record(sequence_input):
            return [sequence_input]
        if isinstance(sequence_input, Path):
            return list(get_record_iterator(sequence_input))
        recs = _records(sequence_input)
        if recs is None:
            raise ValueError(
                "Invalid sequence input, must be a Seq object, a list of Seq objects, a"
                " SeqIO FastaIterator, a SeqIO FastqPhredIterator, or a Path object to a"
                " fasta/fastq file")
        return recs

    def _doc_labels(self) -> list[str]:
        """Result label of every doc column of the hit matrix."""
        return list(self.index.doc_names)

    def _labels(self, display_name: bool) -> list[str]:
        names = self._doc_labels()
        if not display_name:
            return names
        # reference :299-308: "<key> -<display name minus the model name>"
        return [f"{key} -{self.display_names.get(key, 'Unknown').replace(self.model_display_name, '', 1)}"
                for key in names]

    def _doc_mask(self, exclude_ids) -> np.ndarray | None:
        if not exclude_ids:
            return None
        return np.array([name not in exclude_ids for name in self._doc_labels()], dtype=np.uint8)

    def predict_columnar(self, sequence_input, exclude_ids: list[str] = None, step: int = 1,
                         display_name: bool = False) -> MatrixResult:
        """The prediction as a MatrixResult: the same numbers as predict() without
        per-read dictionaries; MatrixResult.save writes the same JSON."""
        ids, _, hits_m, nk = self._matrix(sequence_input, step)
        return MatrixResult(self.slug(), ids, self._labels(display_name), hits_m, nk,
                            sparse_sampling_step=step, doc_mask=self._doc_mask(exclude_ids))

    def predict(self, sequence_input, exclude_ids: list[str] = None, step: int = 1,
                display_name: bool = False, validation: bool = False) -> ModelResult:
        """ModelResult of a record / list / iterator / FASTA-FASTQ path (reference :237-331)."""
        if validation:
            # misclassification detection maps reads with minimap2 against NCBI
            # downloads (:508-601): outside the probe path, see DESIGN.md.
            raise NotImplementedError("validation (alignment-based misclassification detection) "
                                      "is outside the GPU probe path")
        return self.predict_columnar(sequence_input, exclude_ids, step, display_name).to_model_result()

    def detecting_misclassification(self, hits: dict, seq_records: list, min_reads: int = 10) -> dict:
        """Reference :508-601 maps the reads with minimap2 against genomes it
        downloads from NCBI: network and an aligner, outside the k-mer × filter
        path.  Present so a caller switching classes gets this
        error rather than an AttributeError."""
        raise NotImplementedError("detecting_misclassification (minimap2 against NCBI downloads) "
                                  "is outside the GPU probe path")

    # ------------------------------------------------------------ k-mer counts
    def _count_kmers_len(self, length: int, step: int) -> int:
        return math.ceil((length - self.k + 1) / step)   # reference :462

    def _count_kmers(self, sequence_input, step: int = 1) -> int:
        """Total sampled k-mers of a sequence / record / list / iterator (:411-469)."""
        if is_record(sequence_input):
            return self._count_kmers_len(len(seq_text(sequence_input.seq)), step)
        if isinstance(sequence_input, (str, bytes)) or type(sequence_input).__name__ == "Seq":
            return self._count_kmers_len(len(seq_text(sequence_input)), step)
        if isinstance(sequence_input, (list, tuple)) or hasattr(sequence_input, "__next__"):
            total = 0
            for s in sequence_input:
                text = seq_text(s.seq) if is_record(s) else seq_text(s)
                total += self._count_kmers_len(len(text), step)
            return total
        raise ValueError(
            "Invalid sequence input, must be a Seq object, a list of Seq objects, a"
            " SeqIO FastaIterator, or a SeqIO FastqPhredIterator")

    # ------------------------------------------------------------ persistence
    def save(self) -> None:
        json_path = self.base_path / f"{self.slug()}.json"
        (self.base_path / self.slug()).mkdir(exist_ok=True, parents=True)
        json_path.write_text(json.dumps(self.to_dict(), indent=4), encoding="utf-8")

    @staticmethod
    def load(path: Path, docs: tuple[int, int] | None = None) -> "ProbabilisticFilterModel":
        """Reference :351-391.  docs=(lo, hi): only those docs of the bank resident
        (one rank's slice of a docs-sharded bank, distributed.load_docs_slice)."""
        meta = json.loads(Path(path).read_text(encoding="utf-8"))
        model = ProbabilisticFilterModel(
            meta["k"], meta["model_display_name"], meta["author"], meta["author_email"],
            meta["model_type"], Path(path).parent, meta["fpr"], meta["num_hashes"],
            meta["training_accessions"])
        model.display_names = meta["display_names"]
        model._open_index(docs)
        return model

    def _open_index(self, docs: tuple[int, int] | None = None) -> None:
        index_path = Path(self.get_cobs_index_path())
        if not index_path.exists():
            raise FileNotFoundError(f"Index file not found at {index_path}")
        self.index = Bank.open(index_path, XS_BANK_COBS_CLASSIC, device=self.device, docs=docs)

    def close(self) -> None:
        if self.index is not None:
            self.index.close()
            self.index = None


def _stack(parts: list, D: int) -> tuple[np.ndarray, np.ndarray]:
    """Hit rows and k-mer counts of consecutive batches as one matrix (no copy
    for a single batch; batches of different widths widen to the widest)."""
    if not parts:
        return np.zeros((0, D), dtype=np.uint8), np.zeros(0, dtype=np.uint64)
    if len(parts) == 1:
        return parts[0]
    dt = max((h.dtype for h, _ in parts), key=lambda t: t.itemsize)
    # into a recycled host block (bank._HostPool): no fresh pages to fault in now or unmap when the
    # result is dropped (the batches' own arrays go back to the pool once this returns)
    from .bank import _HOST_POOL
    out = _HOST_POOL.empty((sum(h.shape[0] for h, _ in parts), D), dt)
    np.concatenate([h.astype(dt, copy=False) for h, _ in parts], out=out)
    return out, np.concatenate([n for _, n in parts])


def _batches(lens: list[int]) -> Iterable[tuple[int, int]]:
    """Split reads into C-ABI calls of bounded size (reads are never split)."""
    lo, size = 0, 0
    for i, n in enumerate(lens):
        if i > lo and (size + n > MAX_BATCH_BYTES or i - lo >= MAX_BATCH_READS):
            yield lo, i
            lo, size = i, 0
        size += n
    if lo < len(lens):
        yield lo, len(lens)
