"""The Transform graph artifact (`transform_fn/` + `transformed_metadata/`) and its loader.

Reference: `tft.TFTransformOutput(hparams.transform_output)` and
`transform_raw_features(...)` reused at serving/eval (`airflow-dags/taxi_utils.py:211-212,244-245`).
The artifact holds the recorded analyzer constants (`transform_fn/state.json`) and a copy of the
user module whose `preprocessing_fn` replays them.
"""
from __future__ import annotations

import hashlib
import importlib.util
import os
import shutil
import sys

import numpy as np

from .api import TransformState, apply


def import_module_file(path: str, fn_name: str | None = None):
    path = os.path.abspath(path)
    name = "mifx_user_" + hashlib.sha1(path.encode()).hexdigest()[:12]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    if fn_name is not None:
        if not hasattr(mod, fn_name):
            raise AttributeError(f"{path} does not define {fn_name}()")
        return getattr(mod, fn_name)
    return mod


TRANSFORM_FN_DIR = "transform_fn"
TRANSFORMED_METADATA_DIR = "transformed_metadata"


def write_transform_output(out_dir: str, state: TransformState, module_file: str, fn_name: str = "preprocessing_fn",
                           transformed_schema_text: str | None = None, raw_schema_text: str | None = None) -> None:
    fd = os.path.join(out_dir, TRANSFORM_FN_DIR)
    os.makedirs(fd, exist_ok=True)
    with open(os.path.join(fd, "state.json"), "w") as f:
        f.write(state.to_json())
    shutil.copyfile(module_file, os.path.join(fd, "module.py"))
    with open(os.path.join(fd, "fn_name"), "w") as f:
        f.write(fn_name)
    for e in state.entries:  # vocabulary files (tft writes one asset per vocab_filename)
        if e["kind"] == "vocabulary" and e["params"].get("vocab_filename"):
            with open(os.path.join(fd, e["params"]["vocab_filename"]), "w") as f:
                f.write("\n".join(e["values"]) + "\n")
    md = os.path.join(out_dir, TRANSFORMED_METADATA_DIR)
    os.makedirs(md, exist_ok=True)
    if transformed_schema_text:
        with open(os.path.join(md, "schema.pbtxt"), "w") as f:
            f.write(transformed_schema_text)
    if raw_schema_text:
        with open(os.path.join(fd, "raw_schema.pbtxt"), "w") as f:
            f.write(raw_schema_text)


class TransformOutput:
    def __init__(self, transform_output_dir: str):
        self.dir = transform_output_dir
        fd = os.path.join(transform_output_dir, TRANSFORM_FN_DIR)
        with open(os.path.join(fd, "state.json")) as f:
            self.state = TransformState.from_json(f.read())
        with open(os.path.join(fd, "fn_name")) as f:
            fn_name = f.read().strip()
        self.module_path = os.path.join(fd, "module.py")
        self.preprocessing_fn = import_module_file(self.module_path, fn_name)

    def raw_feature_names(self) -> list[str]:
        p = os.path.join(self.dir, TRANSFORM_FN_DIR, "raw_schema.pbtxt")
        if not os.path.exists(p):
            return []
        from ..data_validation import load_schema_text

        return load_schema_text(p).feature_names()

    def transform_raw_features(self, raw_features: dict) -> dict:
        """Apply the recorded transform. Raw features absent at serving time (e.g. the label,
        which the serving receiver drops) are fed as all-missing columns; outputs derived only
        from them are meaningless and ignored by the model signature."""
        feats = {k: np.asarray(v) if not isinstance(v, np.ndarray) else v for k, v in raw_features.items()}
        n = len(next(iter(feats.values()))) if feats else 0
        for name in self.raw_feature_names():
            if name not in feats:
                feats[name] = np.array([None] * n, dtype=object)
        return apply(self.preprocessing_fn, feats, self.state)

    def transformed_schema(self):
        from ..data_validation import load_schema_text

        return load_schema_text(os.path.join(self.dir, TRANSFORMED_METADATA_DIR, "schema.pbtxt"))

    def transformed_feature_spec(self) -> dict:
        return self.transformed_schema().as_feature_spec()

    def vocabulary_by_name(self, vocab_filename: str) -> list[str]:
        for e in self.state.entries:
            if e["kind"] == "vocabulary" and e["params"].get("vocab_filename") == vocab_filename:
                return list(e["values"])
        raise KeyError(vocab_filename)

    def vocabulary_size_by_name(self, vocab_filename: str) -> int:
        return len(self.vocabulary_by_name(vocab_filename))
