"""Sequence filtering over the GPU models (mirror of ``src/xspect/filter_sequences.py``).

``filter_species`` (``:12-68``) and ``filter_genus`` (``:71-124``) predict every
input file, optionally save the classification, take the read ids whose score
for the given label passes the threshold (``ModelResult.
get_filtered_subsequence_labels``, ``result.py:92-149``) and write those records
to a FASTA file (``file_io.filter_sequences``, ``file_io.py:166-191``).  Same
arguments, printed messages, output names and bytes as the reference; the
prediction is the columnar one (``predict_columnar``: one batched GPU probe
per reader window, no per-read dictionaries), the masks are computed over the
hit matrix (``MatrixResult.get_filter_mask``) and the FASTA is written by the
native writer in Bio.SeqIO's layout.
"""
from __future__ import annotations

from pathlib import Path

import numpy as np

from .file_io import prepare_input_output_paths, read_batches


def filter_sequences(input_file: Path, output_file: Path, included_ids: list[str]) -> None:
    """Records of `input_file` whose id is in `included_ids`, in file order, as
    FASTA (``file_io.py:166-191``: every record with a listed id, repeats
    included; no file at all for an empty list)."""
    if not included_ids:
        print("No IDs provided, no output file will be created.")
        return
    wanted = set(included_ids)
    written = 0
    for b in read_batches(Path(input_file)):
        idx = np.fromiter((i for i, rid in enumerate(b.ids()) if rid in wanted), dtype=np.uint32)
        if idx.size:
            b.write_fasta(Path(output_file), idx, append=written > 0)
            written += int(idx.size)
    if not written:  # the reference opens the file for writing before it reads
        Path(output_file).write_text("", encoding="utf-8")


def _filter(model, label: str, input_path: Path, output_path: Path, threshold: float,
            classification_output_path: Path | None, step: int, what: str) -> None:
    input_paths, get_output_path = prepare_input_output_paths(Path(input_path))
    for idx, current_path in enumerate(input_paths):
        result = model.predict_columnar(current_path, step=step)
        result.input_source = current_path.name
        if classification_output_path:
            cls_out = get_output_path(idx, Path(classification_output_path))
            result.save(cls_out)
            print(f"Saved classification results from {current_path.name} as {cls_out.name}")
        included_ids = result.get_filtered_subsequence_labels(label, threshold)
        if not included_ids:
            print(f"No sequences found for the given {what} in {current_path.name}.")
            continue
        filter_output_path = get_output_path(idx, Path(output_path))
        filter_sequences(current_path, filter_output_path, included_ids)
        print(f"Saved filtered sequences from {current_path.name} as {filter_output_path.name}")


def filter_species(model_genus: str, model_species: str, input_path: Path, output_path: Path,
                   threshold: float, classification_output_path: Path | None = None,
                   sparse_sampling_step: int = 1) -> None:
    """Reads whose score for species `model_species` passes `threshold` (-1:
    the species scores highest) under the genus's species model
    (``filter_sequences.py:12-68``; the reference loads it as
    ProbabilisticFilterSVMModel, so the saved classification carries the SVM
    prediction)."""
    from .classify import species_model_path
    from .probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    model = ProbabilisticFilterSVMModel.load(species_model_path(model_genus))
    try:
        _filter(model, model_species, input_path, output_path, threshold, classification_output_path,
                sparse_sampling_step, "species")
    finally:
        model.close()


def filter_genus(model_genus: str, input_path: Path, output_path: Path, threshold: float,
                 classification_output_path: Path | None = None, sparse_sampling_step: int = 1) -> None:
    """Reads whose genus score passes `threshold` under the genus Bloom model
    (``filter_sequences.py:71-124``)."""
    from .classify import genus_model_path
    from .probabilistic_single_filter_model import ProbabilisticSingleFilterModel

    model = ProbabilisticSingleFilterModel.load(genus_model_path(model_genus))
    try:
        _filter(model, model_genus, input_path, output_path, threshold, classification_output_path,
                sparse_sampling_step, "genus")
    finally:
        model.close()
