"""Species model with an SVM over the total-score vector.

Drop-in for ``xspect.models.probabilistic_filter_svm_model.ProbabilisticFilterSVMModel``
(reference ``src/xspect/models/probabilistic_filter_svm_model.py:22-315``).
The SVM input vector is ``[round(T_d / N, 2) for d in sorted(labels)]``
(``:211-213`` with ``result.py:57-72``); T_d and N are integer sums of the GPU
hit matrix, so the vector is bit-exact with the CPU path.  The SVC itself
(fit from scores.csv on every call, ``:225-274``) stays scikit-learn on CPU.
"""
from __future__ import annotations

import csv
import json
from pathlib import Path

from .file_io import FASTA_ENDINGS, FASTQ_ENDINGS
from .probabilistic_filter_model import ProbabilisticFilterModel
from .result import MatrixResult, ModelResult


def svm_training_files(svm_path: Path) -> list[tuple[Path, Path]]:
    """(species folder, genome file) pairs in the reference's walk order:
    ``svm_path.iterdir()`` then each folder's ``iterdir()``, unsorted
    (probabilistic_filter_svm_model.py:147-152), so scores.csv rows come out
    in the reference's order."""
    out = []
    for species_folder in svm_path.iterdir():
        if not species_folder.is_dir():
            continue
        for file in species_folder.iterdir():
            if file.suffix[1:] not in FASTA_ENDINGS + FASTQ_ENDINGS:
                continue
            out.append((species_folder, file))
    return out


class ProbabilisticFilterSVMModel(ProbabilisticFilterModel):
    """COBS species bank on the GPU + scikit-learn SVC on the score vector."""

    def __init__(self, k: int, model_display_name: str, author: str | None,
                 author_email: str | None, model_type: str, base_path: Path, kernel: str,
                 c: float, fpr: float = 0.01, num_hashes: int = 7,
                 training_accessions: dict[str, list[str]] | None = None,
                 svm_accessions: dict[str, list[str]] | None = None) -> None:
        super().__init__(k=k, model_display_name=model_display_name, author=author,
                         author_email=author_email, model_type=model_type, base_path=base_path,
                         fpr=fpr, num_hashes=num_hashes, training_accessions=training_accessions)
        self.kernel = kernel
        self.c = c
        self.svm_accessions = svm_accessions

    def to_dict(self) -> dict:
        return super().to_dict() | {"kernel": self.kernel, "C": self.c,
                                    "svm_accessions": self.svm_accessions}

    def set_svm_params(self, kernel: str, c: float) -> None:
        self.kernel = kernel
        self.c = c
        self.save()

    def scores_csv_path(self) -> Path:
        return self.base_path / self.slug() / "scores.csv"

    def fit(self, dir_path: Path, svm_path: Path, display_names: dict[str, str] | None = None,
            svm_step: int = 1, training_accessions: dict[str, list[str]] | None = None,
            svm_accessions: dict[str, list[str]] | None = None) -> None:
        """Build the bank, then score every SVM training genome with the base
        predict (reference :107-173) and write scores.csv."""
        super().fit(dir_path, display_names=display_names, training_accessions=training_accessions)
        self.svm_accessions = svm_accessions
        rows = []
        for species_folder, file in svm_training_files(svm_path):
            print(f"Calculating {file.name} scores for SVM training...")
            totals = ProbabilisticFilterModel.predict_columnar(self, file, step=svm_step).get_total_scores()
            values = ",".join(str(v) for _, v in sorted(totals.items()))
            rows.append(f"{file.stem},{values},{species_folder.name}")
        header = f"file,{','.join(sorted(self.display_names))},label_id"
        self.scores_csv_path().parent.mkdir(parents=True, exist_ok=True)
        self.scores_csv_path().write_text("\n".join([header] + rows), encoding="utf-8")

    @staticmethod
    def svm_vector(result: ModelResult) -> list[float]:
        """Total scores sorted by label: the SVM feature row of one input."""
        return [v for _, v in sorted(result.get_scores()["total"].items())]

    def predict_columnar(self, sequence_input, exclude_ids: list[str] = None, step: int = 1,
                         display_name: bool = False) -> MatrixResult:
        """Columnar prediction; the SVM label comes from the total scores only (:208-223)."""
        res = super().predict_columnar(sequence_input, exclude_ids, step, display_name)
        features = [[v for _, v in sorted(res.get_total_scores().items())]]
        res.prediction = str(self._get_svm(exclude_ids).predict(features)[0])
        return res

    def predict(self, sequence_input, exclude_ids: list[str] = None, step: int = 1,
                display_name: bool = False, validation: bool = False) -> ModelResult:
        if validation:
            raise NotImplementedError("validation (alignment-based misclassification detection) "
                                      "is outside the GPU probe path")
        return self.predict_columnar(sequence_input, exclude_ids, step, display_name).to_model_result()

    def _get_svm(self, exclude_ids):
        """SVC(kernel, C) fitted on scores.csv minus excluded labels/columns (:225-274)."""
        from sklearn.svm import SVC

        keys = list(self.display_names.keys())
        drop = {i for i, key in enumerate(keys) if exclude_ids is not None and key in exclude_ids}
        x_train, y_train = [], []
        with open(self.scores_csv_path(), "r", encoding="utf-8") as fh:
            fh.readline()
            for row in csv.reader(fh):
                label = row[-1]
                if exclude_ids is not None and label in exclude_ids:
                    continue
                feats = row[1:-1]
                x_train.append([float(v) for i, v in enumerate(feats) if i not in drop])
                y_train.append(label)
        svm = SVC(kernel=self.kernel, C=self.c)
        svm.fit(x_train, y_train)
        return svm

    @staticmethod
    def load(path: Path, docs: tuple[int, int] | None = None) -> "ProbabilisticFilterSVMModel":
        meta = json.loads(Path(path).read_text(encoding="utf-8"))
        model = ProbabilisticFilterSVMModel(
            meta["k"], meta["model_display_name"], meta["author"], meta["author_email"],
            meta["model_type"], Path(path).parent, meta["kernel"], meta["C"], fpr=meta["fpr"],
            num_hashes=meta["num_hashes"], training_accessions=meta["training_accessions"],
            svm_accessions=meta["svm_accessions"])
        model.display_names = meta["display_names"]
        model._open_index(docs)
        return model
