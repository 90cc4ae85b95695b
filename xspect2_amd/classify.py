"""Classification entry points over the GPU models (mirror of ``src/xspect/classify.py``).

Model files are found where XspecT keeps them (``definitions.py:10-46``,
``model_management.py:27-77``): ``<root>/models/<slug>.json`` with
``<root>`` = ``~/xspect-data`` or ``./xspect-data`` (or ``$XSPECT_DATA``).
"""
from __future__ import annotations

import json
import os
from pathlib import Path

from .file_io import prepare_input_output_paths
from .util import slugify


def xspect_root() -> Path:
    env = os.environ.get("XSPECT_DATA")
    if env:
        return Path(env)
    home = Path.home() / "xspect-data"
    if home.exists():
        return home
    cwd = Path.cwd() / "xspect-data"
    if cwd.exists():
        return cwd
    home.mkdir(parents=True, exist_ok=True)
    return home


def model_dir() -> Path:
    p = xspect_root() / "models"
    p.mkdir(parents=True, exist_ok=True)
    return p


def genus_model_path(genus: str) -> Path:
    return model_dir() / (slugify(genus) + "-genus.json")


def species_model_path(genus: str) -> Path:
    return model_dir() / (slugify(genus) + "-species.json")


def mlst_model_path(organism: str, scheme: str) -> Path:
    return model_dir() / (slugify(organism + "-" + scheme + "-mlst") + ".json")


def is_svm_model(model_json: Path) -> bool:
    if not model_json.exists():
        raise ValueError(f"Model at {model_json} does not exist.")
    return json.loads(model_json.read_text(encoding="utf-8")).get("model_class") == \
        "ProbabilisticFilterSVMModel"


class _SaveBehind:
    """Results of a directory's files saved on one worker thread while the
    next file is predicted (the JSON of a 1 M-read file takes ~0.6 s of host
    writing, its prediction ~0.08 s on the GPU).  One save at a time, in file
    order; "Saved result as ..." is printed when a save has finished, and a
    failed save raises from the next submit() or from finish()."""

    def __init__(self):
        from concurrent.futures import ThreadPoolExecutor
        self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="xs-save")
        self._pending = None

    def _wait(self) -> None:
        if self._pending is not None:
            pending, self._pending = self._pending, None
            print(f"Saved result as {pending.result()}")  # result() re-raises the save's exception

    def submit(self, result, path: Path) -> None:
        self._wait()

        def save():
            result.save(path)
            return path.name
        self._pending = self._pool.submit(save)

    def finish(self) -> None:
        try:
            self._wait()
        finally:
            self._pool.shutdown(wait=True)


def classify_genus(model_genus: str, input_path: Path, output_path: Path, step: int = 1):
    from .probabilistic_single_filter_model import ProbabilisticSingleFilterModel

    model = ProbabilisticSingleFilterModel.load(genus_model_path(model_genus))
    saver = _SaveBehind()
    try:
        inputs, out_path = prepare_input_output_paths(Path(input_path))
        for idx, current in enumerate(inputs):
            # columnar result: same JSON as ModelResult.save, no per-read dicts
            result = model.predict_columnar(current, step=step)
            result.input_source = current.name
            saver.submit(result, out_path(idx, Path(output_path)))
    finally:
        try:
            saver.finish()
        finally:
            model.close()  # the filter's HBM goes back now, not at garbage collection (a serving process)


def classify_species(model_genus: str, input_path: Path, output_path: Path, step: int = 1,
                     display_name: bool = False, validation: bool = False,
                     exclude_ids: list[str] | None = None):
    from .probabilistic_filter_model import ProbabilisticFilterModel
    from .probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    path = species_model_path(model_genus)
    cls = ProbabilisticFilterSVMModel if is_svm_model(path) else ProbabilisticFilterModel
    model = cls.load(path)
    saver = _SaveBehind()
    try:
        inputs, out_path = prepare_input_output_paths(Path(input_path))
        for idx, current in enumerate(inputs):
            if validation:
                result = model.predict(current, exclude_ids=exclude_ids, step=step,
                                       display_name=display_name, validation=validation)
            else:
                # columnar result: same JSON as ModelResult.save, no per-read dicts
                result = model.predict_columnar(current, exclude_ids=exclude_ids, step=step,
                                                display_name=display_name)
            result.input_source = current.name
            saver.submit(result, out_path(idx, Path(output_path)))
    finally:
        try:
            saver.finish()
        finally:
            model.close()


def classify_species_sharded(model_genus: str, input_path: Path, output_path: Path, step: int = 1,
                             display_name: bool = False, exclude_ids: list[str] | None = None):
    """``classify_species`` over the ranks of an initialised torch.distributed
    process group (one process per GPU, ``torchrun``; BASELINE config 3):
    every rank loads the model (its bank on ``LOCAL_RANK``), classifies its
    byte range of each input file, the D+1 totals are all-reduced over RCCL,
    rank 0 forms the SVM label, and every rank writes its JSON shard
    (``distributed.shard_path`` of the reference's output name;
    ``distributed.merge_result_shards`` gives the single-process JSON)."""
    from . import distributed
    from .probabilistic_filter_model import ProbabilisticFilterModel
    from .probabilistic_filter_svm_model import ProbabilisticFilterSVMModel

    path = species_model_path(model_genus)
    cls = ProbabilisticFilterSVMModel if is_svm_model(path) else ProbabilisticFilterModel
    model = cls.load(path)
    try:
        inputs, out_path = prepare_input_output_paths(Path(input_path))
        outs = []
        for idx, current in enumerate(inputs):
            target = out_path(idx, Path(output_path))
            distributed.classify_species_sharded(model, current, target, step=step, display_name=display_name,
                                                 exclude_ids=exclude_ids)
            outs.append(target)
    finally:
        model.close()
    return outs


def classify_mlst(input_path: Path, organism: str, mlst_scheme: str, output_path: Path,
                  limit: bool):
    from .probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel

    model = ProbabilisticFilterMlstSchemeModel.load(mlst_model_path(organism, mlst_scheme))
    try:
        inputs, out_path = prepare_input_output_paths(Path(input_path))
        for idx, current in enumerate(inputs):
            result = model.predict(current, step=1, limit=limit)
            result.input_source = current.name
            path = out_path(idx, Path(output_path))
            result.save(path)
            print(f"Saved result as {path.name}")
    finally:
        model.close()


def classify_pipeline(model_genus: str, input_path: Path, output_dir: Path | None = None, threshold: float = 0.7,
                      sparse_sampling_step: int = 1, display_names: bool = False, validation: bool = False,
                      mlst_scheme: str | None = None):
    """The full pipeline of ``xspect`` (``src/xspect/main.py:84-187`` all_pipeline):
    genus filter, species classification, MLST for A. baumannii, as one fused
    GPU pass per input file (xspect2_amd.pipeline).  ``mlst_scheme`` names the
    abaumannii scheme (the reference takes the first one it has downloaded)."""
    from .pipeline import run_pipeline
    from .probabilistic_filter_model import ProbabilisticFilterModel
    from .probabilistic_filter_svm_model import ProbabilisticFilterSVMModel
    from .probabilistic_single_filter_model import ProbabilisticSingleFilterModel

    if validation:
        raise NotImplementedError("validation (alignment-based misclassification detection) "
                                  "is outside the GPU probe path")
    genus = ProbabilisticSingleFilterModel.load(genus_model_path(model_genus))
    spath = species_model_path(model_genus)
    species = (ProbabilisticFilterSVMModel if is_svm_model(spath) else ProbabilisticFilterModel).load(spath)
    mlst = None
    if mlst_scheme is not None:
        from .probabilistic_filter_mlst_model import ProbabilisticFilterMlstSchemeModel
        p = mlst_model_path("abaumannii", mlst_scheme)
        if p.exists():
            mlst = ProbabilisticFilterMlstSchemeModel.load(p)
    try:
        return run_pipeline(genus, species, Path(input_path), output_dir, threshold, sparse_sampling_step,
                            display_names, mlst=mlst)
    finally:
        for m in (genus, species, mlst):
            if m is not None:
                m.close()
