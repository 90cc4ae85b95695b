"""Fused genus -> species classification.

The reference pipeline (``src/xspect/main.py:93-160``) makes three passes over
the data:
  1. ``filter_genus`` (``filter_sequences.py:71-124``): parse the input,
     predict with the genus Bloom model, save the genus classification and
     write the records whose genus score passes the threshold to a filtered
     FASTA (``file_io.py:166-191``);
  2. ``classify_species`` on the filtered directory: parse the FASTA again and
     predict with the species model;
  3. MLST on the filtered files when a species prediction is "470".

Here one parse feeds both models.  Every batch of the native reader goes to
the GPU once.  The genus probe runs there, and only its per-read hits and
k-mer counts come back (12 B per read).  The keep decision is
``round(h / n, 2) >= threshold`` (``result.py`` ``get_filter_mask``), made on
the host with Python's own rounding over the batch's distinct (h, n) pairs.
The kept reads are then compacted on the device (``xs_gather_reads_device``)
and probed against the species bank.  Outputs are the reference's files, with
the same names and the same bytes:
``genus_classification_<run>.json``,
``filtered_sequences/genus_filtered_<run>.fasta`` and
``species_classification_<run>_<i>.json``.
"""
from __future__ import annotations

import os
import uuid
from pathlib import Path

import numpy as np

from .bank import gather_reads_device
from .file_io import FASTA_ENDINGS, FASTQ_ENDINGS, prepare_input_output_paths, read_batches
from .result import MatrixResult


def check_threshold(threshold: float) -> None:
    """result.py get_filter_mask's range check."""
    if threshold < 0 and not threshold == -1 or threshold > 1:
        raise ValueError("The filter threshold must be between 0 and 1.")


def keep_mask(hits: np.ndarray, num_kmers: np.ndarray, threshold: float) -> np.ndarray:
    """Reads whose single-label score round(h / n, 2) passes `threshold`
    (-1: the label is the maximum, which a one-label result always is).

    Python's round is applied to every distinct (h, n) pair, so the decision is
    exactly the reference's (numpy's rounding differs on some halves)."""
    check_threshold(threshold)
    h = np.asarray(hits, dtype=np.uint64).reshape(-1)
    n = np.asarray(num_kmers, dtype=np.uint64).reshape(-1)
    if threshold == -1 or h.size == 0:
        return np.ones(h.size, dtype=bool)
    key = (h << np.uint64(32)) | n
    uniq, inv = np.unique(key, return_inverse=True)
    ok = np.fromiter((round(int(k >> 32) / int(k & 0xFFFFFFFF), 2) >= threshold for k in uniq.tolist()),
                     dtype=bool, count=uniq.size)
    return ok[inv]


class _Collector:
    """Per-file columnar pieces of one model's result."""

    def __init__(self):
        self.ids, self.hits, self.nk = [], [], []

    def add(self, ids, hits, nk):
        self.ids += ids
        self.hits.append(hits)
        self.nk.append(nk)

    def result(self, slug, labels, step, **kw) -> MatrixResult:
        D = len(labels)
        hits = np.concatenate(self.hits) if self.hits else np.zeros((0, D), dtype=np.uint32)
        nk = np.concatenate(self.nk) if self.nk else np.zeros(0, dtype=np.uint64)
        return MatrixResult(slug, self.ids, labels, hits.reshape(-1, D), nk, sparse_sampling_step=step, **kw)


def _partial(fasta_out: Path) -> Path:
    """Where a file's filtered FASTA is written until its pass completes (its
    name ends in no FASTA/FASTQ ending, so a directory glob never sees it)."""
    return fasta_out.with_name(fasta_out.name + ".partial")


def _short_read_error() -> ValueError:
    return ValueError("Invalid sequence, must be longer than k")


def _fused_file(path: Path, genus, species, threshold: float, step: int, fasta_out: Path,
                batch_bytes: int | None, display_names: bool):
    """One parse of `path`: genus result (all reads), species result (kept
    reads), filtered FASTA.  Returns (genus MatrixResult, species MatrixResult
    or None, records written, species error or None).

    Side effects follow the reference's order (main.py:93-160): genus predict
    covers the whole file before anything is written, so a read of length
    <= genus.k raises with no filtered FASTA left behind; the filtered FASTA
    is complete before species predict runs, so a kept read of length
    <= species.k does not stop the genus pass or the FASTA - its ValueError is
    returned and raised by run_pipeline where classify_species would raise it."""
    partial = _partial(fasta_out)
    try:
        gres, sres, written, serr = _fused_pass(path, genus, species, threshold, step, partial, batch_bytes,
                                                display_names)
    except BaseException:
        partial.unlink(missing_ok=True)
        raise
    if written:
        os.replace(partial, fasta_out)
    return gres, sres, written, serr


def _fused_pass(path: Path, genus, species, threshold: float, step: int, fasta_out: Path,
                batch_bytes: int | None, display_names: bool):
    import torch

    gbank, sbank = genus.bf, species.index
    if gbank is None or sbank is None:
        raise ValueError("The model has not been trained yet")
    dev = torch.device("cuda", gbank.info.device)
    stream = torch.cuda.current_stream(dev)
    s = stream.cuda_stream
    D = sbank.num_docs
    gcol, scol = _Collector(), _Collector()
    written = 0
    serr = None
    for b in read_batches(path, batch_bytes, pinned=True):
        L = b.lengths()
        if (L <= genus.k).any():  # genus predict on every read (:224-225)
            raise _short_read_error()
        n = b.n
        nbytes = int(b.packed.offsets[-1])
        d_seq = torch.from_numpy(b.packed.buf[:max(nbytes, 1)]).to(dev, non_blocking=True)
        d_off = torch.from_numpy(b.packed.offsets.view(np.int64)).to(dev, non_blocking=True)
        d_gh = torch.empty(n, dtype=torch.int32, device=dev)
        d_gnk = torch.empty(n, dtype=torch.int64, device=dev)
        gbank.query_device(d_seq, nbytes, d_off, n, step, d_gh, d_gnk, None, stream=s)
        gh = d_gh.cpu().numpy().view(np.uint32)
        gnk = d_gnk.cpu().numpy().view(np.uint64)
        ids = b.ids()
        gcol.add(ids, gh.reshape(n, 1), gnk)
        keep = keep_mask(gh, gnk, threshold)
        idx = np.flatnonzero(keep).astype(np.uint32)
        m = int(idx.size)
        if not m:
            continue
        fasta_out.parent.mkdir(parents=True, exist_ok=True)
        b.write_fasta(fasta_out, idx, append=written > 0)
        written += m
        if serr is None and (L[idx] <= species.k).any():  # species predict on the kept reads
            serr = _short_read_error()
        if serr is not None:
            continue
        out_off = np.zeros(m + 1, dtype=np.uint64)
        np.cumsum(L[idx], out=out_off[1:])
        mbytes = int(out_off[-1])
        d_idx = torch.from_numpy(idx.view(np.int32)).to(dev)
        d_off2 = torch.from_numpy(out_off.view(np.int64)).to(dev)
        d_seq2 = torch.empty(max(mbytes, 1), dtype=torch.uint8, device=dev)
        gather_reads_device(d_seq, d_off, d_idx, m, d_seq2, d_off2, stream=s)
        d_sh = torch.empty((m, D), dtype=torch.int32, device=dev)
        d_snk = torch.empty(m, dtype=torch.int64, device=dev)
        sbank.query_device(d_seq2, mbytes, d_off2, m, step, d_sh, d_snk, None, stream=s)
        sh = d_sh.cpu().numpy().view(np.uint32)
        snk = d_snk.cpu().numpy().view(np.uint64)
        scol.add([ids[i] for i in idx.tolist()], sh, snk)
    gres = gcol.result(genus.slug(), genus._labels(False), step)
    if len(set(gres.ids)) != len(gcol.ids):
        # duplicate read ids: the reference filters by id over the whole file
        # (record.id in included_ids); redo the hand-off with that rule
        return _by_id_fallback(path, genus, species, gres, threshold, step, fasta_out, batch_bytes,
                               display_names)
    sres = None
    if written and serr is None:
        sres = scol.result(species.slug(), species._labels(display_names), step)
    return gres, sres, written, serr


def _by_id_fallback(path, genus, species, gres, threshold, step, fasta_out, batch_bytes, display_names):
    """Filter by id over the whole file (record.id in included_ids), as
    file_io.py:188-191 does, when read ids repeat."""
    from .packing import pack_sequences

    included = {rid for rid, keep in zip(gres.ids, keep_mask(gres.hits[:, 0], gres.num_kmers, threshold)) if keep}
    written = 0
    serr = None
    scol = _Collector()
    for b in read_batches(path, batch_bytes):
        ids = b.ids()
        idx = np.array([i for i, rid in enumerate(ids) if rid in included], dtype=np.uint32)
        if not idx.size:
            continue
        fasta_out.parent.mkdir(parents=True, exist_ok=True)
        b.write_fasta(fasta_out, idx, append=written > 0)
        written += int(idx.size)
        if serr is None and (b.lengths()[idx] <= species.k).any():
            serr = _short_read_error()
        if serr is not None:
            continue
        raw = b.packed.buf
        o = b.packed.offsets
        seqs = [raw[o[i]:o[i + 1]].tobytes() for i in idx.tolist()]
        h, nk = species.index.query(pack_sequences(seqs), step=step)
        scol.add([ids[i] for i in idx.tolist()], h, nk)
    sres = scol.result(species.slug(), species._labels(display_names), step) if written and serr is None else None
    return gres, sres, written, serr


def _svm_predict(species, sres: MatrixResult) -> None:
    if hasattr(species, "_get_svm") and sres is not None:
        feats = [[v for _, v in sorted(sres.get_total_scores().items())]]
        sres.prediction = str(species._get_svm(None).predict(feats)[0])


def run_pipeline(genus, species, input_path: Path, output_dir: Path | None = None, threshold: float = 0.7,
                 step: int = 1, display_names: bool = False, run_id: str | None = None, mlst=None,
                 batch_bytes: int | None = None, log=print) -> dict:
    """Genus filter + species classification (+ MLST for "470") in one pass per
    input file, writing the reference pipeline's outputs (main.py:93-187).

    `genus`: a ProbabilisticSingleFilterModel; `species`: a
    ProbabilisticFilterModel or ProbabilisticFilterSVMModel; `mlst`: an optional
    ProbabilisticFilterMlstSchemeModel for step 3.  Returns the output paths."""
    check_threshold(threshold)
    run_id = run_id or str(uuid.uuid4())
    output_dir = Path(output_dir or f"xspect_results_{run_id}")
    output_dir.mkdir(exist_ok=True, parents=True)
    filtered_dir = output_dir / "filtered_sequences"
    filtered_dir.mkdir(exist_ok=True, parents=True)
    genus_filtered = filtered_dir / f"genus_filtered_{run_id}.fasta"
    genus_cls = output_dir / f"genus_classification_{run_id}.json"
    species_cls = output_dir / f"species_classification_{run_id}.json"
    out = {"run_id": run_id, "genus": [], "filtered": [], "species": [], "mlst": []}

    # step 1 (+ the species probe of the kept reads, same pass)
    log(f"Step 1/3: Filtering for genus {genus.model_display_name}...")
    inputs, get_out = prepare_input_output_paths(Path(input_path))
    species_of: dict[Path, MatrixResult | ValueError] = {}
    for idx, current in enumerate(inputs):
        fasta_out = get_out(idx, genus_filtered)
        gres, sres, written, serr = _fused_file(current, genus, species, threshold, step, fasta_out, batch_bytes,
                                          display_names)
        gres.input_source = current.name
        cls_out = get_out(idx, genus_cls)
        gres.save(cls_out)
        out["genus"].append(cls_out)
        log(f"Saved classification results from {current.name} as {cls_out.name}")
        if not written:
            log(f"No sequences found for the given genus in {current.name}.")
            continue
        species_of[fasta_out.resolve()] = sres if serr is None else serr
        out["filtered"].append(fasta_out)
        log(f"Saved filtered sequences from {current.name} as {fasta_out.name}")

    filtered_files = [p for e in FASTA_ENDINGS + FASTQ_ENDINGS for p in filtered_dir.glob(f"*.{e}")]
    if not filtered_files:
        log("No sequences passed the genus filter. Pipeline aborted.")
        return out

    # step 2: species results of every file in the filtered directory, named as
    # classify_species names them for a directory input
    log(f"Step 2/3: Classifying species for {len(filtered_files)} filtered file(s)...")
    finputs, fget_out = prepare_input_output_paths(filtered_dir)
    predictions = []
    for idx, f in enumerate(finputs):
        sres = species_of.get(f.resolve())
        if isinstance(sres, ValueError):  # species predict of this file raises here (classify.py:78-92)
            raise sres
        if sres is None:  # a file of an earlier run in the same directory
            sres = species.predict_columnar(f, step=step, display_name=display_names)
        else:
            _svm_predict(species, sres)
        sres.input_source = f.name
        path = fget_out(idx, species_cls)
        sres.save(path)
        out["species"].append(path)
        predictions.append(sres.prediction)
        log(f"Saved result as {path.name}")

    # step 3: MLST when a species prediction is A. baumannii (470)
    if "470" in predictions and mlst is not None:
        log("Step 3/3: Running MLST classification for abaumannii...")
        mlst_out = output_dir / f"mlst_classification_{run_id}.json"
        for idx, f in enumerate(finputs):
            res = mlst.predict(f, step=1, limit=False)
            res.input_source = f.name
            path = fget_out(idx, mlst_out)
            res.save(path)
            out["mlst"].append(path)
    elif "470" in predictions:
        log("Warning: No MLST schemes available for abaumannii. Skipping MLST classification.")
    else:
        log("Step 3/3: Not running MLST classification (organism is not Acinetobacter baumannii).")
    return out


def reference_pipeline(genus, species, input_path: Path, output_dir: Path, threshold: float = 0.7,
                       step: int = 1, display_names: bool = False, run_id: str = "ref", log=print) -> dict:
    """The reference's three-pass flow on the same models (predict, filter by id,
    write FASTA, re-parse), for comparison and tests."""
    check_threshold(threshold)
    output_dir = Path(output_dir)
    filtered_dir = output_dir / "filtered_sequences"
    filtered_dir.mkdir(exist_ok=True, parents=True)
    genus_filtered = filtered_dir / f"genus_filtered_{run_id}.fasta"
    genus_cls = output_dir / f"genus_classification_{run_id}.json"
    species_cls = output_dir / f"species_classification_{run_id}.json"
    inputs, get_out = prepare_input_output_paths(Path(input_path))
    out = {"genus": [], "filtered": [], "species": []}
    for idx, current in enumerate(inputs):
        result = genus.predict_columnar(current, step=step)
        result.input_source = current.name
        result.save(get_out(idx, genus_cls))
        out["genus"].append(get_out(idx, genus_cls))
        label = genus._labels(False)[0]
        included = set(result.to_model_result().get_filtered_subsequence_labels(label, threshold))
        if not included:
            continue
        fasta_out = get_out(idx, genus_filtered)
        written = 0
        for b in read_batches(current):
            keep = np.array([i for i, rid in enumerate(b.ids()) if rid in included], dtype=np.uint32)
            if keep.size:
                b.write_fasta(fasta_out, keep, append=written > 0)
                written += int(keep.size)
        out["filtered"].append(fasta_out)
    finputs, fget_out = prepare_input_output_paths(filtered_dir)
    for idx, f in enumerate(finputs):
        res = species.predict_columnar(f, step=step, display_name=display_names)
        res.input_source = f.name
        res.save(fget_out(idx, species_cls))
        out["species"].append(fget_out(idx, species_cls))
    return out
