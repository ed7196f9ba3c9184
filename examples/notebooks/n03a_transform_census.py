"""Notebook 03a (TensorFlow Transform, advanced) with mifx: the census income pipeline
(reference `notebooks/03a_TensorFlow_Transform_Advanced.ipynb` cells 9-28).

  raw adult.data / adult.test lines -> fix ", " separators (+ trailing '.' on test labels)
  -> MapAndFilterErrors(decode) with a bad-record counter
  -> analyze + transform (scale_to_0_1 numerics, densified optional education-num, one
     vocabulary per categorical feature written as a vocab file, label lookup ['>50K','<=50K'])
  -> transformed TFRecords + transform_fn directory
  -> LinearClassifier (numeric columns + vocabulary-file categorical columns, FTRL, summed
     sigmoid cross-entropy as TF1 canned estimators) trained for TRAIN_NUM_EPOCHS
  -> export with a serving function that applies the transform to RAW features, and evaluate.

The census zip is downloaded by the notebook; offline, synthetic rows in the same format are
generated. `WEB_TEST_BROWSER` shrinks the run exactly as the notebook's test shortcut does."""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import mifx.transform as tft  # noqa: E402
from mifx.io.tfrecord import encode_example, read_tfrecords, decode_example, write_tfrecords  # noqa: E402
from mifx.trainer.optim import Ftrl  # noqa: E402

CATEGORICAL_FEATURE_KEYS = ["workclass", "education", "marital-status", "occupation", "relationship", "race", "sex",
                            "native-country"]
NUMERIC_FEATURE_KEYS = ["age", "capital-gain", "capital-loss", "hours-per-week"]
OPTIONAL_NUMERIC_FEATURE_KEYS = ["education-num"]
LABEL_KEY = "label"
ORDERED_COLUMNS = ["age", "workclass", "fnlwgt", "education", "education-num", "marital-status", "occupation",
                   "relationship", "race", "sex", "capital-gain", "capital-loss", "hours-per-week", "native-country",
                   "label"]

if os.getenv("WEB_TEST_BROWSER", False):
    TRAIN_NUM_EPOCHS, NUM_TRAIN_INSTANCES, TRAIN_BATCH_SIZE, NUM_TEST_INSTANCES = 1, 1, 1, 1
else:
    TRAIN_NUM_EPOCHS, NUM_TRAIN_INSTANCES, TRAIN_BATCH_SIZE, NUM_TEST_INSTANCES = 16, 32561, 128, 16281

TRANSFORMED_TRAIN_DATA_FILEBASE = "train_transformed"
TRANSFORMED_TEST_DATA_FILEBASE = "test_transformed"
EXPORTED_MODEL_DIR = "exported_model_dir"


# ------------------------------------------------------------------------------ data
def synthesize_census(path: str, n: int, seed: int, test: bool = False, bad_rows: int = 3) -> None:
    """adult.data-format lines with a learnable income signal (offline stand-in for census.zip)."""
    rng = np.random.default_rng(seed)
    vocab = {"workclass": ["Private", "Self-emp-not-inc", "Local-gov", "State-gov", "Federal-gov", "?"],
             "education": ["HS-grad", "Some-college", "Bachelors", "Masters", "Doctorate", "11th"],
             "marital-status": ["Married-civ-spouse", "Never-married", "Divorced", "Widowed"],
             "occupation": ["Prof-specialty", "Craft-repair", "Exec-managerial", "Adm-clerical", "Sales", "?"],
             "relationship": ["Husband", "Not-in-family", "Own-child", "Unmarried", "Wife"],
             "race": ["White", "Black", "Asian-Pac-Islander", "Other"],
             "sex": ["Male", "Female"], "native-country": ["United-States", "Mexico", "India", "Germany", "?"]}
    edu_num = {"HS-grad": 9, "Some-college": 10, "Bachelors": 13, "Masters": 14, "Doctorate": 16, "11th": 7}
    lines = ["|1x3 Cross validator"] if test else []
    for _ in range(n):
        r = {k: vocab[k][int(rng.integers(len(v)))] for k, v in vocab.items()}
        age, hours = int(rng.integers(17, 80)), int(rng.integers(10, 70))
        gain = int(rng.exponential(800)) if rng.random() < 0.1 else 0
        loss = int(rng.exponential(300)) if rng.random() < 0.05 else 0
        score = (0.05 * (age - 40) + 0.04 * (hours - 40) + 0.3 * (edu_num[r["education"]] - 10)
                 + (1.0 if r["marital-status"] == "Married-civ-spouse" else -0.8) + gain / 2000.0
                 + rng.normal(0, 0.8))
        label = ">50K" if score > 0.8 else "<=50K"
        vals = [age, r["workclass"], int(rng.integers(20000, 500000)), r["education"], edu_num[r["education"]],
                r["marital-status"], r["occupation"], r["relationship"], r["race"], r["sex"], gain, loss, hours,
                r["native-country"], label + ("." if test else "")]
        lines.append(", ".join(str(v) for v in vals))
    for i in range(bad_rows):  # malformed records -> counted and dropped by MapAndFilterErrors
        lines.insert(1 + i * 7, "this, is, not, a, census, row")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


class MapAndFilterErrors:
    """Like map(fn) but drops elements whose fn raises, counting them (Beam metric
    `census_example:bad_elements` in the notebook)."""

    def __init__(self, fn):
        self.fn = fn
        self.bad_elements = 0

    def __call__(self, elements):
        for e in elements:
            try:
                yield self.fn(e)
            except Exception:  # noqa: BLE001 - the notebook's broad catch
                self.bad_elements += 1


def decode_csv_line(line: str) -> dict:
    parts = line.split(",")
    if len(parts) != len(ORDERED_COLUMNS):
        raise ValueError(f"expected {len(ORDERED_COLUMNS)} fields, got {len(parts)}")
    rec = dict(zip(ORDERED_COLUMNS, parts))
    for k in NUMERIC_FEATURE_KEYS:
        rec[k] = float(rec[k])
    rec["education-num"] = float(rec["education-num"]) if rec["education-num"] != "" else None
    return rec


def read_raw(path: str, test: bool, counter: MapAndFilterErrors) -> dict:
    with open(path) as f:
        lines = [ln.rstrip("\n") for ln in f if ln.strip()]
    if test:
        lines = lines[1:]  # skip_header_lines=1
    lines = [ln.replace(", ", ",") for ln in lines]
    if test:
        lines = [ln[:-1] for ln in lines]  # RemoveTrailingPeriods
    recs = list(counter(lines))
    return {k: np.array([r[k] for r in recs], dtype=object if k not in NUMERIC_FEATURE_KEYS else np.float32)
            for k in ORDERED_COLUMNS}


# --------------------------------------------------------------------------- transform
def preprocessing_fn(inputs):
    outputs = dict(inputs)
    for key in NUMERIC_FEATURE_KEYS:
        outputs[key] = tft.scale_to_0_1(outputs[key])
    for key in OPTIONAL_NUMERIC_FEATURE_KEYS:  # sparse_to_dense(default 0) then scale
        dense = tft.fill_in_missing(outputs[key], 0.0)
        outputs[key] = tft.scale_to_0_1(dense)
    for key in CATEGORICAL_FEATURE_KEYS:
        tft.vocabulary(inputs[key], vocab_filename=key)
    outputs[LABEL_KEY] = tft.apply_vocabulary(outputs[LABEL_KEY], [">50K", "<=50K"], default_value=-1)
    outputs.pop("fnlwgt", None)
    return outputs


def _write_examples(path: str, cols: dict) -> int:
    n = len(cols[LABEL_KEY])
    recs = (encode_example({k: [v[i].item() if hasattr(v[i], "item") else v[i]] for k, v in cols.items()})
            for i in range(n))
    return write_tfrecords(path, recs)


def transform_data(train_file: str, test_file: str, working_dir: str) -> dict:
    os.makedirs(working_dir, exist_ok=True)
    counter = MapAndFilterErrors(decode_csv_line)
    raw_train = read_raw(train_file, False, counter)
    transformed, state = tft.analyze(preprocessing_fn, raw_train)
    _write_examples(os.path.join(working_dir, TRANSFORMED_TRAIN_DATA_FILEBASE), transformed)
    raw_test = read_raw(test_file, True, counter)
    transformed_test = tft.apply(preprocessing_fn, raw_test, state)
    _write_examples(os.path.join(working_dir, TRANSFORMED_TEST_DATA_FILEBASE), transformed_test)
    tft.write_transform_output(working_dir, state, os.path.abspath(__file__))
    return {"bad_elements": counter.bad_elements, "train": len(raw_train[LABEL_KEY]), "test": len(raw_test[LABEL_KEY])}


# ------------------------------------------------------------------------------ model
class LinearClassifier(torch.nn.Module):
    """Numeric columns + categorical_column_with_vocabulary_file columns (OOV -> no weight)."""

    def __init__(self, vocab_sizes: list[int]):
        super().__init__()
        self.num = torch.nn.Parameter(torch.zeros(len(NUMERIC_FEATURE_KEYS)))
        self.offsets = torch.tensor([0] + list(np.cumsum(vocab_sizes)[:-1]), dtype=torch.long)
        self.cat = torch.nn.Parameter(torch.zeros(int(sum(vocab_sizes))))
        self.bias = torch.nn.Parameter(torch.zeros(()))

    def forward(self, num: torch.Tensor, cat_ids: torch.Tensor) -> torch.Tensor:
        valid = cat_ids >= 0
        idx = (cat_ids.clamp_min(0) + self.offsets.to(cat_ids.device)).flatten()
        w = self.cat.index_select(0, idx).view_as(cat_ids) * valid
        return num @ self.num + w.sum(1) + self.bias


def _features(cols: dict, vocabs: dict, dev) -> tuple[torch.Tensor, torch.Tensor]:
    num = torch.tensor(np.stack([np.asarray(cols[k], np.float32) for k in NUMERIC_FEATURE_KEYS], 1), device=dev)
    ids = np.stack([_lookup(cols[k], vocabs[k]) for k in CATEGORICAL_FEATURE_KEYS], 1)
    return num, torch.tensor(ids, dtype=torch.long, device=dev)


def _lookup(values, vocab: list[str]) -> np.ndarray:
    table = {v: i for i, v in enumerate(vocab)}
    return np.array([table.get(str(v), -1) for v in values], dtype=np.int64)


def _read_examples(path: str) -> dict:
    rows = [decode_example(b) for b in read_tfrecords(path)]
    out = {}
    for k in rows[0]:
        vals = [r[k][0] for r in rows]
        out[k] = np.array([v.decode() if isinstance(v, bytes) else v for v in vals], dtype=object)
    return out


def train_and_evaluate(working_dir: str, num_train_instances: int = NUM_TRAIN_INSTANCES,
                       num_test_instances: int = NUM_TEST_INSTANCES, epochs: int = TRAIN_NUM_EPOCHS,
                       batch_size: int = TRAIN_BATCH_SIZE, device=None) -> dict:
    dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
    tfo = tft.TransformOutput(working_dir)
    vocabs = {k: tfo.vocabulary_by_name(k) for k in CATEGORICAL_FEATURE_KEYS}
    train = _read_examples(os.path.join(working_dir, TRANSFORMED_TRAIN_DATA_FILEBASE))
    test = _read_examples(os.path.join(working_dir, TRANSFORMED_TEST_DATA_FILEBASE))
    model = LinearClassifier([len(vocabs[k]) for k in CATEGORICAL_FEATURE_KEYS]).to(dev)
    opt = Ftrl(model.parameters(), lr=min(0.2, 1 / np.sqrt(len(NUMERIC_FEATURE_KEYS) + len(CATEGORICAL_FEATURE_KEYS))))
    num, ids = _features(train, vocabs, dev)
    y = torch.tensor(train[LABEL_KEY].astype(np.float32), device=dev)
    n = min(len(y), num_train_instances)
    steps = max(1, epochs * n // batch_size)
    g = torch.Generator(device="cpu").manual_seed(0)
    for step in range(steps):
        idx = torch.randint(0, n, (batch_size,), generator=g).to(dev)
        opt.zero_grad()
        loss = torch.nn.functional.binary_cross_entropy_with_logits(model(num[idx], ids[idx]), y[idx],
                                                                    reduction="sum")
        loss.backward()
        opt.step()
    tnum, tids = _features(test, vocabs, dev)
    ty = torch.tensor(test[LABEL_KEY].astype(np.float32), device=dev)[:num_test_instances]
    with torch.no_grad():
        logits = model(tnum[:num_test_instances], tids[:num_test_instances])
        acc = float(((logits > 0).float() == ty).float().mean())
        avg_loss = float(torch.nn.functional.binary_cross_entropy_with_logits(logits, ty))
    export_dir = os.path.join(working_dir, EXPORTED_MODEL_DIR, "1")
    os.makedirs(export_dir, exist_ok=True)
    torch.save({k: v.cpu() for k, v in model.state_dict().items()}, os.path.join(export_dir, "model.pt"))
    with open(os.path.join(export_dir, "signature.json"), "w") as f:
        json.dump({"transform_output": os.path.abspath(working_dir),
                   "vocab_sizes": [len(vocabs[k]) for k in CATEGORICAL_FEATURE_KEYS]}, f)
    return {"accuracy": acc, "average_loss": avg_loss, "global_step": steps, "export_dir": export_dir}


def serve(export_dir: str, raw_rows: list[dict]) -> np.ndarray:
    """Serving input fn: RAW features (no label) -> transform_raw_features -> model -> P(label=1)."""
    with open(os.path.join(export_dir, "signature.json")) as f:
        sig = json.load(f)
    tfo = tft.TransformOutput(sig["transform_output"])
    raw = {k: np.array([r.get(k) for r in raw_rows], dtype=object) for k in ORDERED_COLUMNS if k != LABEL_KEY}
    for k in NUMERIC_FEATURE_KEYS:
        raw[k] = raw[k].astype(np.float32)
    raw[LABEL_KEY] = np.array([""] * len(raw_rows), dtype=object)
    feats = tfo.transform_raw_features(raw)
    model = LinearClassifier(sig["vocab_sizes"])
    model.load_state_dict(torch.load(os.path.join(export_dir, "model.pt"), weights_only=True))
    vocabs = {k: tfo.vocabulary_by_name(k) for k in CATEGORICAL_FEATURE_KEYS}
    num, ids = _features(feats, vocabs, "cpu")
    with torch.no_grad():
        return torch.sigmoid(model(num, ids)).numpy()


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "mifx_census"))
    ap.add_argument("--train_rows", type=int, default=32561)
    ap.add_argument("--test_rows", type=int, default=16281)
    ap.add_argument("--epochs", type=int, default=TRAIN_NUM_EPOCHS)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    os.makedirs(a.workdir, exist_ok=True)
    train_file, test_file = os.path.join(a.workdir, "adult.data"), os.path.join(a.workdir, "adult.test")
    synthesize_census(train_file, a.train_rows, 0)
    synthesize_census(test_file, a.test_rows, 1, test=True)
    info = transform_data(train_file, test_file, os.path.join(a.workdir, "working"))
    print("transform:", info)
    res = train_and_evaluate(os.path.join(a.workdir, "working"), epochs=a.epochs, device=a.device)
    print("evaluation:", res)
    probe = decode_csv_line("39,State-gov,77516,Bachelors,13,Never-married,Adm-clerical,Not-in-family,White,Male,"
                            "2174,0,40,United-States,<=50K")
    print("serving P(<=50K) for a raw example:", float(serve(res["export_dir"], [probe])[0]))
    return {**info, **res}


if __name__ == "__main__":
    main()
