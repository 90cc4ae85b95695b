"""ModelResult: per-read hit dictionaries -> scores, totals, masks, JSON.

Behavioural mirror of the reference class
(``src/xspect/models/result.py:7-189``); pinned by
``tests/golden/model_result_vectors.json`` (outputs of the reference class).
"""
from __future__ import annotations

import ctypes
import json
from json import dumps
from pathlib import Path

import numpy as np

from .packing import PackedIds


class ModelResult:
    """Hits per subsequence and label, plus the k-mer count of each subsequence."""

    def __init__(
        self,
        model_slug: str,
        hits: dict[str, dict[str, int]],
        num_kmers: dict[str, int],
        sparse_sampling_step: int = 1,
        prediction: str | None = None,
        input_source: str | None = None,
    ):
        # result.py:33-36 — "total" is the reserved key of get_scores()
        if "total" in hits:
            raise ValueError("'total' is a reserved key and cannot be used as a subsequence")
        self.model_slug = model_slug
        self.hits = hits
        self.num_kmers = num_kmers
        self.sparse_sampling_step = sparse_sampling_step
        self.prediction = prediction
        self.input_source = input_source
        # result.py:43 — validation output travels under "misclassified"
        self.misclassified = self.hits.pop("misclassified", None)

    def get_scores(self) -> dict:
        """round(hits / num_kmers, 2) per subsequence and label, plus "total"."""
        out: dict = {}
        for sub, per_label in self.hits.items():
            n = self.num_kmers[sub]
            out[sub] = {label: round(v / n, 2) for label, v in per_label.items()}
        n_all = sum(self.num_kmers.values())
        out["total"] = {label: round(v / n_all, 2) for label, v in self.get_total_hits().items()}
        return out

    def get_total_hits(self) -> dict[str, int]:
        """Hits per label summed over subsequences (labels of the first subsequence)."""
        first = next(iter(self.hits.values())) if self.hits else None
        if first is None:
            # the reference indexes list(self.hits.values())[0] here
            raise IndexError("list index out of range")
        totals = dict.fromkeys(first, 0)
        for per_label in self.hits.values():
            for label, v in per_label.items():
                totals[label] += v
        return totals

    def get_filter_mask(self, label: str, filter_threshold: float) -> dict[str, bool]:
        """Subsequences whose score for `label` passes the threshold (-1 = argmax)."""
        if filter_threshold < 0 and not filter_threshold == -1 or filter_threshold > 1:
            raise ValueError("The filter threshold must be between 0 and 1.")
        scores = self.get_scores()
        scores.pop("total")
        if filter_threshold == -1:
            return {sub: s[label] == max(s.values()) for sub, s in scores.items()}
        return {sub: s[label] >= filter_threshold for sub, s in scores.items()}

    def get_filtered_subsequence_labels(self, label: str, filter_threshold: float = 0.7) -> list[str]:
        return [sub for sub, keep in self.get_filter_mask(label, filter_threshold).items() if keep]

    def to_dict(self) -> dict:
        res = {
            "model_slug": self.model_slug,
            "sparse_sampling_step": self.sparse_sampling_step,
            "hits": self.hits,
            "scores": self.get_scores(),
            "num_kmers": self.num_kmers,
            "misclassified": self.misclassified,
            "input_source": self.input_source,
        }
        if self.prediction is not None:
            res["prediction"] = self.prediction
        return res

    def save(self, path: Path) -> None:
        path = Path(path)
        path.parent.mkdir(exist_ok=True, parents=True)
        path.write_text(dumps(self.to_dict(), indent=4), encoding="utf-8")


def _json_packed(strings: list[str]) -> tuple[bytes, np.ndarray]:
    """JSON string literals (json.dumps, ensure_ascii) of `strings`, packed + offsets."""
    enc = [json.dumps(s).encode("ascii") for s in strings]
    off = np.zeros(len(enc) + 1, dtype=np.uint64)
    if enc:
        np.cumsum(np.fromiter(map(len, enc), dtype=np.uint64, count=len(enc)), out=off[1:])
    return b"".join(enc), off


def cobs_order(row: np.ndarray, docs: np.ndarray) -> np.ndarray:
    """`docs` in COBS result order for one hit row: count descending, ties by doc index."""
    return docs[np.argsort(-row[docs].astype(np.int64), kind="stable")]


class MatrixResult:
    """Columnar ModelResult: read ids, labels, an n x D hit
    matrix and per-read k-mer counts, as the probe produces them.

    It holds the numbers ModelResult holds as per-read dictionaries
    (``src/xspect/models/result.py:7-189``): ``to_model_result()`` builds those
    dictionaries, and ``save()`` writes the same JSON bytes as
    ``ModelResult.save`` without them: the per-read sections are formatted
    natively (xs_write_result_sections), so 10^6-read results take seconds.
    Per-read labels follow COBS result order (count descending, ties by doc
    index); ``doc_mask`` drops excluded docs (predict's exclude_ids).
    Duplicate read ids collapse as they do in the reference's dictionaries:
    the first position, the last record's values.  ``ids`` may be a
    ``PackedIds`` (the reader's id buffer, as ``predict_columnar`` of a file
    passes it): no Python string per read is made unless a caller reads one.

    ``hits`` may be uint8 / uint16 / uint32: a matrix narrowed on the device
    (counts never exceed a read's k-mer count) is kept narrow, and widened
    only where a caller reads values.  ``set_job_totals`` makes the result one
    shard of a read-sharded job: its "total" scores (and get_total_hits) are
    the whole job's, all-reduced over the ranks (xspect2_amd.distributed).
    """

    def __init__(self, model_slug: str, ids: list[str] | PackedIds, labels: list[str], hits: np.ndarray,
                 num_kmers: np.ndarray, sparse_sampling_step: int = 1, prediction: str | None = None,
                 input_source: str | None = None, doc_mask: np.ndarray | None = None):
        if "total" in ids:
            raise ValueError("'total' is a reserved key and cannot be used as a subsequence")
        hits = np.ascontiguousarray(hits)
        if hits.dtype not in (np.uint8, np.uint16, np.uint32):
            hits = hits.astype(np.uint32)
        num_kmers = np.ascontiguousarray(num_kmers, dtype=np.uint64)
        if hits.ndim != 2 or hits.shape[0] != len(ids) or hits.shape[1] != len(labels) or \
                num_kmers.shape != (len(ids),):
            raise ValueError("hits must be [len(ids), len(labels)] and num_kmers [len(ids)]")
        packed = isinstance(ids, PackedIds)
        if (ids.has_duplicates() if packed else len(set(ids)) != len(ids)):
            ids = list(ids)
            last = {rid: i for i, rid in enumerate(ids)}
            first_order = list(dict.fromkeys(ids))
            rows = np.array([last[rid] for rid in first_order], dtype=np.int64)
            ids, hits, num_kmers = first_order, hits[rows], num_kmers[rows]
        self.model_slug = model_slug
        self.ids = ids if isinstance(ids, PackedIds) else list(ids)
        self.labels = list(labels)
        self.hits = hits
        self.num_kmers = num_kmers
        self.sparse_sampling_step = sparse_sampling_step
        self.prediction = prediction
        self.input_source = input_source
        self.doc_mask = None if doc_mask is None else np.ascontiguousarray(doc_mask, dtype=np.uint8)
        self.misclassified = None
        self.job_total_hits: np.ndarray | None = None    # whole-job sums (a shard of a sharded job)
        self.job_total_kmers: int | None = None
        self.job_order_row: np.ndarray | None = None     # the job's first hit row (orders "total")

    def set_job_totals(self, total_hits: np.ndarray, total_kmers: int, order_row: np.ndarray) -> None:
        """Make this result one shard of a read-sharded job: "total" covers the
        job (per-doc sums and k-mer count over every rank, labels in the COBS
        order of the job's first read), the per-read sections this shard's reads."""
        self.job_total_hits = np.ascontiguousarray(total_hits, dtype=np.uint64)
        self.job_total_kmers = int(total_kmers)
        self.job_order_row = np.ascontiguousarray(order_row, dtype=np.uint32)

    @property
    def docs(self) -> np.ndarray:
        d = np.arange(len(self.labels))
        return d if self.doc_mask is None else d[self.doc_mask.astype(bool)]

    def _needs_dicts(self) -> bool:
        # reference quirks outside the columnar writer: a read called
        # "misclassified" is popped from the hits (result.py:43), equal labels collapse
        return "misclassified" in self.ids or len(set(self.labels)) != len(self.labels)

    def to_model_result(self) -> ModelResult:
        docs = self.docs
        hits = {}
        for i, rid in enumerate(self.ids):
            row = self.hits[i]
            order = cobs_order(row, docs).tolist()
            hits[rid] = {self.labels[d]: int(row[d]) for d in order}
        nk = {rid: int(n) for rid, n in zip(self.ids, self.num_kmers.tolist())}
        return ModelResult(self.model_slug, hits, nk, self.sparse_sampling_step, self.prediction,
                           self.input_source)

    def get_total_hits(self) -> dict[str, int]:
        if self.job_total_hits is not None:
            tot, first = self.job_total_hits, self.job_order_row
        elif not self.ids:
            raise IndexError("list index out of range")
        else:
            tot, first = self.hits.sum(axis=0, dtype=np.uint64), self.hits[0]
        return {self.labels[d]: int(tot[d]) for d in cobs_order(first, self.docs).tolist()}

    def get_total_scores(self) -> dict[str, float]:
        """get_scores()["total"] without the per-read part."""
        n_all = self.job_total_kmers if self.job_total_hits is not None else int(self.num_kmers.sum())
        return {label: round(v / n_all, 2) for label, v in self.get_total_hits().items()}

    def get_filter_mask(self, label: str, filter_threshold: float) -> dict[str, bool]:
        """ModelResult.get_filter_mask (result.py:92-123) over the matrix:
        {read id: round(h / n, 2) >= threshold} for `label`'s column, or with
        threshold -1 whether `label`'s rounded score is the read's largest.
        Python's round is applied to each distinct (h, n) pair, so every
        decision is the reference's."""
        if filter_threshold < 0 and not filter_threshold == -1 or filter_threshold > 1:
            raise ValueError("The filter threshold must be between 0 and 1.")
        if self._needs_dicts():
            return self.to_model_result().get_filter_mask(label, filter_threshold)
        if not self.ids:
            raise IndexError("list index out of range")  # get_scores -> get_total_hits, as the reference
        docs = self.docs.tolist()
        col = next((d for d in docs if self.labels[d] == label), None)
        if col is None:
            raise KeyError(label)  # score[label] in the reference
        n = self.num_kmers.astype(np.uint64)
        h = self.hits[:, col].astype(np.uint64)
        if filter_threshold == -1:
            hmax = self.hits[:, self.docs].max(axis=1).astype(np.uint64)
            keys = np.concatenate([(h << np.uint64(32)) | n, (hmax << np.uint64(32)) | n])
        else:
            keys = (h << np.uint64(32)) | n
        uniq, inv = np.unique(keys, return_inverse=True)
        score = np.fromiter((round(int(k >> 32) / int(k & 0xFFFFFFFF), 2) for k in uniq.tolist()),
                            dtype=np.float64, count=uniq.size)[inv]
        m = len(self.ids)
        keep = score[:m] == score[m:] if filter_threshold == -1 else score >= filter_threshold
        return dict(zip(self.ids, keep.tolist()))

    def get_filtered_subsequence_labels(self, label: str, filter_threshold: float = 0.7) -> list[str]:
        """ModelResult.get_filtered_subsequence_labels (result.py:125-149)."""
        return [rid for rid, keep in self.get_filter_mask(label, filter_threshold).items() if keep]

    def best(self) -> tuple[np.ndarray, np.ndarray]:
        """(best doc or XS_BEST_AMBIGUOUS, max hits) per read, over the kept docs."""
        docs = self.docs
        sub = self.hits[:, docs]
        m = sub.max(axis=1) if docs.size else np.zeros(len(self.ids), dtype=np.uint32)
        ties = (sub == m[:, None]).sum(axis=1) if docs.size else np.zeros(len(self.ids))
        arg = docs[sub.argmax(axis=1)] if docs.size else np.zeros(len(self.ids), dtype=np.int64)
        best = np.where(ties == 1, arg, 0xFFFFFFFF).astype(np.uint32)
        return best, m.astype(np.uint32)

    def save(self, path: Path) -> None:
        """Write the JSON ModelResult.save writes (byte-identical)."""
        path = Path(path)
        shard = self.job_total_hits is not None
        if self._needs_dicts():
            mr = self.to_model_result()
            if not shard:
                return mr.save(path)
            # the shard's own reads, the job's "total" (no local get_total_hits:
            # a shard may hold no reads)
            scores = {sub: {lab: round(v / mr.num_kmers[sub], 2) for lab, v in per.items()}
                      for sub, per in mr.hits.items()}
            scores["total"] = self.get_total_scores()
            d = {"model_slug": mr.model_slug, "sparse_sampling_step": mr.sparse_sampling_step, "hits": mr.hits,
                 "scores": scores, "num_kmers": mr.num_kmers, "misclassified": mr.misclassified,
                 "input_source": mr.input_source}
            if mr.prediction is not None:
                d["prediction"] = mr.prediction
            path.parent.mkdir(exist_ok=True, parents=True)
            path.write_text(dumps(d, indent=4), encoding="utf-8")
            return None
        if not self.ids and not shard:
            raise IndexError("list index out of range")  # get_total_hits on no reads, as the reference
        from ._lib import check, load
        path.parent.mkdir(exist_ok=True, parents=True)
        head = "{\n    %s: %s,\n    %s: %s,\n    " % (
            dumps("model_slug"), dumps(self.model_slug), dumps("sparse_sampling_step"),
            dumps(self.sparse_sampling_step))
        path.write_text(head, encoding="utf-8")
        ids_b, ids_off = self.ids.json_packed() if isinstance(self.ids, PackedIds) else _json_packed(self.ids)
        lab_b, lab_off = _json_packed(self.labels)
        mask = self.doc_mask
        vp = ctypes.c_void_p
        check(load().xs_write_result_sections(
            str(path).encode(), len(self.ids), len(self.labels), vp(self.hits.ctypes.data), self.hits.itemsize,
            vp(self.num_kmers.ctypes.data), ids_b, vp(ids_off.ctypes.data), lab_b, vp(lab_off.ctypes.data),
            vp(mask.ctypes.data) if mask is not None else None,
            vp(self.job_total_hits.ctypes.data) if shard else None, self.job_total_kmers if shard else 0,
            vp(self.job_order_row.ctypes.data) if shard else None, 0))
        tail = [("misclassified", self.misclassified), ("input_source", self.input_source)]
        if self.prediction is not None:
            tail.append(("prediction", self.prediction))
        body = ",\n    ".join(f"{dumps(k)}: {dumps(v, indent=4)}" for k, v in tail)
        with open(path, "a", encoding="utf-8") as fh:
            fh.write("    " + body + "\n}")

    def save_npz(self, path: Path) -> None:
        """Columnar dump: ids, labels, hits, num_kmers (+ mask, metadata)."""
        np.savez(path, ids=np.array(self.ids, dtype=object).astype(str), labels=np.array(self.labels).astype(str),
                 hits=self.hits, num_kmers=self.num_kmers,
                 doc_mask=self.doc_mask if self.doc_mask is not None else np.ones(len(self.labels), np.uint8),
                 meta=np.array(json.dumps({"model_slug": self.model_slug,
                                           "sparse_sampling_step": self.sparse_sampling_step,
                                           "prediction": self.prediction, "input_source": self.input_source})))

    @staticmethod
    def load_npz(path: Path) -> "MatrixResult":
        z = np.load(path, allow_pickle=False)
        meta = json.loads(str(z["meta"]))
        return MatrixResult(meta["model_slug"], z["ids"].tolist(), z["labels"].tolist(), z["hits"], z["num_kmers"],
                            meta["sparse_sampling_step"], meta["prediction"], meta["input_source"], z["doc_mask"])


class MlstResult:
    """MLST strain-type results (mirror of ``src/xspect/models/mlst_result.py:7-62``)."""

    def __init__(self, scheme_model: str, steps: int, hits: dict[str, list[dict]],
                 input_source: str | None = None):
        self.scheme_model = scheme_model
        self.steps = steps
        self.hits = hits
        self.input_source = input_source

    def get_results(self) -> dict:
        return dict(self.hits.items())

    def to_dict(self) -> dict:
        return {
            "Scheme": self.scheme_model,
            "Steps": self.steps,
            "Results": self.get_results(),
            "Input_source": self.input_source,
        }

    def save(self, output_path: Path | str) -> None:
        output_path = Path(output_path)
        output_path.parent.mkdir(exist_ok=True, parents=True)
        output_path.write_text(dumps(self.to_dict(), indent=4), encoding="utf-8")
