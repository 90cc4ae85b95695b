"""Genus model: one Bloom filter (rbloom semantics) resident in HBM.

Drop-in for ``xspect.models.probabilistic_single_filter_model.ProbabilisticSingleFilterModel``
(reference ``src/xspect/models/probabilistic_single_filter_model.py:16-180``).
The reference walks every k-mer in Python, takes
``min(kmer, str(kmer.reverse_complement()))`` (case preserved, Biopython IUPAC
complement) and calls ``kmer in bf`` — a Rust call that calls back into Python
``xxh3_64_intdigest`` (``:122-124,161-180``).  Here a batch of reads is one
call: canonical k-mer, XXH3-64 and the K index probes all run on the GPU.
"""
from __future__ import annotations

import json
from pathlib import Path

import numpy as np

from ._lib import XS_BANK_RBLOOM
from .bank import Bank, bloom_parameters
from .file_io import check_input_path, is_record, read_batches, seq_text
from .packing import pack_sequences
from .probabilistic_filter_model import ProbabilisticFilterModel


class ProbabilisticSingleFilterModel(ProbabilisticFilterModel):
    """Single-filter (genus) model."""

    def __init__(self, k: int, model_display_name: str, author: str | None,
                 author_email: str | None, model_type: str, base_path: Path, fpr: float = 0.01,
                 training_accessions: list[str] | None = None) -> None:
        super().__init__(k=k, model_display_name=model_display_name, author=author,
                         author_email=author_email, model_type=model_type, base_path=base_path,
                         fpr=fpr, num_hashes=1, training_accessions=training_accessions)
        self.bf: Bank | None = None

    def bloom_path(self) -> Path:
        return self.base_path / self.slug() / "filter.bloom"

    def fit(self, file_path: Path, display_name: str,
            training_accessions: list[str] | None = None) -> None:
        """Bloom(total_length - k + 1, fpr) over every k-mer of the file (:63-96)."""
        self.training_accessions = training_accessions
        check_input_path(file_path)
        total_length = sum(int(b.packed.nbytes) for b in read_batches(file_path))
        nbytes, nhash = bloom_parameters(total_length - self.k + 1, self.fpr)
        bank = Bank.create_bloom(self.k, nbytes, nhash, device=self.device)
        for b in read_batches(file_path):
            bank.build(b.packed)
        self.display_names[file_path.stem] = display_name
        bank.save(self.bloom_path())
        if self.bf is not None:
            self.bf.close()
        self.bf = bank
        self.index = bank

    def calculate_hits(self, sequence, exclude_ids=None, step: int = 1) -> dict:
        """{first display name: number of sampled k-mers in the filter} (:98-125)."""
        if is_record(sequence):
            sequence = sequence.seq
        if not isinstance(sequence, (str, bytes, bytearray)) and type(sequence).__name__ not in ("Seq", "MutableSeq"):
            raise ValueError("Invalid sequence, must be a Bio.Seq object")
        text = seq_text(sequence)
        if not len(text) > self.k:
            raise ValueError("Invalid sequence, must be longer than k")
        hits, _ = self.bf.query(pack_sequences([text]), step=step)
        return {next(iter(self.display_names)): int(hits[0, 0])}

    def _hit_dict(self, row: np.ndarray, exclude_ids) -> dict:
        return {next(iter(self.display_names)): int(row[0])}

    def _doc_labels(self) -> list[str]:
        return [next(iter(self.display_names))]

    def _doc_mask(self, exclude_ids):
        return None  # the genus filter has one label; exclude_ids does not apply

    @staticmethod
    def load(path: Path) -> "ProbabilisticSingleFilterModel":
        meta = json.loads(Path(path).read_text(encoding="utf-8"))
        model = ProbabilisticSingleFilterModel(
            meta["k"], meta["model_display_name"], meta["author"], meta["author_email"],
            meta["model_type"], Path(path).parent, fpr=meta["fpr"],
            training_accessions=meta["training_accessions"])
        model.display_names = meta["display_names"]
        bank = Bank.open(model.bloom_path(), XS_BANK_RBLOOM, device=model.device, term_size=model.k)
        model.bf = bank
        model.index = bank
        return model
