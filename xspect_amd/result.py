"""ModelResult: per-read hit dictionaries -> scores, totals, masks, JSON.

Behavioural mirror of the reference class
(``src/xspect/models/result.py:7-189``); pinned by
``tests/golden/model_result_vectors.json`` (outputs of the reference class).
"""
from __future__ import annotations

from json import dumps
from pathlib import Path


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
