"""Container components of the KFP taxi pipeline, runnable as `python3 -m mifx.kfp_components.taxi <step> ...`.

Reference pipeline: `kubeflow-pipelines/taxi/taxi-cab-classification-pipeline.py:31-133` — eight
steps loaded from component.yaml URLs (tfdv, tft, dnntrainer, tfma, predict, confusion_matrix,
roc, deployer). These are the same steps on this framework: TFDV-equivalent stats/schema/
anomalies, Transform analyze+apply with the user's `preprocess(inputs)` module, the taxi DNN on
the HIP gather/sparse-Adagrad kernels, sliced evaluation, batch prediction, confusion matrix and
ROC (KFP `mlpipeline-ui-metadata.json` / `mlpipeline-metrics.json` outputs), and a deployer that
writes (and optionally applies) the serving manifests for `mifx.serving.server`.

Schema format is the reference's column schema JSON: [{"name": ..., "type": CATEGORY|NUMBER|KEY}]."""
from __future__ import annotations

import argparse
import ast
import csv
import json
import math
import os
import sys

import numpy as np

# ---------------------------------------------------------------------------------------------
# helpers


def _write_output(path: str | None, value) -> None:
    if path:
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        with open(path, "w") as f:
            f.write(str(value))


def _read_csv(path: str, column_names: list | None = None) -> dict:
    """CSV (optionally headerless, with `column_names`) -> {column: np.array(object)} with '' -> None."""
    with open(path, newline="") as f:
        rows = list(csv.reader(f))
    if column_names is None:
        column_names, rows = rows[0], rows[1:]
    cols = {c: [] for c in column_names}
    for r in rows:
        for c, v in zip(column_names, r):
            cols[c].append(v if v != "" else None)
    return {c: np.array(v, dtype=object) for c, v in cols.items()}


def _typed(cols: dict, schema: list) -> dict:
    out = {}
    types = {s["name"]: s["type"] for s in schema}
    for c, v in cols.items():
        t = types.get(c, "CATEGORY")
        if t == "NUMBER":
            out[c] = np.array([np.nan if x is None else float(x) for x in v], dtype=np.float64)
        else:
            out[c] = np.array([None if x is None else str(x) for x in v], dtype=object)
    return out


def _load_columns(path: str, column_names_file: str | None):
    names = None
    if column_names_file:
        with open(column_names_file) as f:
            names = json.load(f)
    return _read_csv(path, names)


_LAMBDA_NAMES = {"float": float, "int": int, "abs": abs, "min": min, "max": max, "round": round, "math": math}
_LAMBDA_NODES = (ast.Expression, ast.Lambda, ast.arguments, ast.arg, ast.Name, ast.Load, ast.Constant, ast.BinOp,
                 ast.UnaryOp, ast.BoolOp, ast.Compare, ast.IfExp, ast.Call, ast.Attribute, ast.Subscript, ast.operator,
                 ast.unaryop, ast.boolop, ast.cmpop, ast.Tuple)


def _compile_target_lambda(src: str):
    """Compile the pipeline's `target_lambda` (e.g. "lambda x: (x['target'] > x['fare'] * 0.2)", the reference's
    taxi-cab-classification-pipeline.py:60 argument) into a function.

    The expression is pipeline-author code, as in the reference (which runs it unchecked). It is parsed with
    `ast` and only a whitelist of expression nodes is accepted: one lambda; names limited to its parameters and
    float / int / abs / min / max / round / math; attributes only on `math` and never dunder; subscripts,
    arithmetic, comparisons, boolean ops and conditional expressions. Anything else (attribute walks such as
    ().__class__, comprehensions, other names) is rejected before evaluation."""
    tree = ast.parse(src.strip(), mode="eval")
    if not isinstance(tree.body, ast.Lambda):
        raise ValueError("target_lambda must be a lambda expression")
    params = {a.arg for a in tree.body.args.args}
    if sum(isinstance(n, ast.Lambda) for n in ast.walk(tree)) != 1:
        raise ValueError("target_lambda: nested lambdas are not allowed")
    for node in ast.walk(tree):
        if not isinstance(node, _LAMBDA_NODES):
            raise ValueError(f"target_lambda: {type(node).__name__} is not allowed")
        if isinstance(node, ast.Name) and node.id not in params and node.id not in _LAMBDA_NAMES:
            raise ValueError(f"target_lambda: name {node.id!r} is not allowed")
        if isinstance(node, ast.Attribute) and (node.attr.startswith("_") or not (
                isinstance(node.value, ast.Name) and node.value.id == "math")):
            raise ValueError(f"target_lambda: attribute {node.attr!r} is not allowed")
    return eval(compile(tree, "<target_lambda>", "eval"), {"__builtins__": {}, **_LAMBDA_NAMES})  # noqa: S307


# ---------------------------------------------------------------------------------------------
# steps


def tfdv(a) -> None:
    """Statistics for the inference and validation data, inferred column schema, anomalies."""
    from ..data_validation import stats as dvstats
    from ..data_validation import validate as dvval
    from ..io import dataset

    train = _load_columns(a.inference_data, a.column_names)
    evald = _load_columns(a.validation_data, a.column_names)
    keys = set(k.strip() for k in (a.key_columns or "").split(",") if k.strip())
    schema = []
    for c, v in train.items():
        nums = [x for x in v if x is not None]
        is_num = bool(nums) and all(_is_number(x) for x in nums)
        kind = "KEY" if c in keys else ("NUMBER" if is_num else "CATEGORY")
        schema.append({"name": c, "type": kind})
    os.makedirs(a.validation_output, exist_ok=True)
    spath = os.path.join(a.validation_output, "schema.json")
    with open(spath, "w") as f:
        json.dump(schema, f, indent=1)
    st_train = dvstats.generate_statistics_from_table(dataset.to_table(_typed(train, schema)), "train")
    st_eval = dvstats.generate_statistics_from_table(dataset.to_table(_typed(evald, schema)), "eval")
    dvstats.write_stats(st_train, os.path.join(a.validation_output, "train_stats.json"))
    inferred = dvval.infer_schema(st_train)
    anomalies = dvval.validate_statistics(st_eval, inferred)
    vpath = os.path.join(a.validation_output, "validation_result.json")
    with open(vpath, "w") as f:
        f.write(anomalies.to_json())
    _write_output(a.schema_out, spath)
    _write_output(a.validation_result_out, vpath)


def _is_number(x) -> bool:
    try:
        float(x)
        return True
    except (TypeError, ValueError):
        return False


def tft(a) -> None:
    """Analyze on the training data, apply to train and eval; write transformed parquet + transform graph."""
    from ..io import dataset
    from ..transform import analyze as t_analyze
    from ..transform import apply as t_apply
    from ..transform.output import import_module_file, write_transform_output

    with open(a.schema) as f:
        schema = json.load(f)
    fn = import_module_file(a.preprocessing_module, "preprocess")
    train = _typed(_read_csv(a.training_data_file_pattern, [s["name"] for s in schema]), schema)
    evald = _typed(_read_csv(a.evaluation_data_file_pattern, [s["name"] for s in schema]), schema)
    out_train, state = t_analyze(fn, train)
    out_eval = t_apply(fn, evald, state)
    os.makedirs(a.transformed_data_dir, exist_ok=True)
    dataset.write_split(os.path.join(a.transformed_data_dir, "train"), out_train)
    dataset.write_split(os.path.join(a.transformed_data_dir, "eval"), out_eval)
    write_transform_output(os.path.join(a.transformed_data_dir, "transform_fn"), state, a.preprocessing_module,
                           "preprocess")
    _write_output(a.transformed_data_dir_out, a.transformed_data_dir)


def dnntrainer(a) -> None:
    """Train the taxi DNN (hidden `hidden_layer_size`, Adagrad) and export a servable model."""
    import torch

    from ..io import dataset
    from ..models.taxi_dnn import TaxiDNN, TaxiDNNConfig, columns_to_tensors
    from ..serving.saved_model import save_module
    from ..trainer.taxi_dnn_trainer import TaxiDNNTrainer

    n_gpus = int(a.num_gpus or 1)
    if n_gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # data parallel: this container step launches one rank per GPU of itself (rank 0 exports)
        from ..trainer.distributed import run_ranks

        run_ranks(["-m", "mifx.kfp_components.taxi"] + list(a._argv), n_gpus,
                  os.path.join(a.training_output_dir, "dp_run"))
        return
    from ..parallel import dist as mdist

    env = mdist.init("gloo" if a.device == "cpu" else None)
    pg = torch.distributed.group.WORLD if env.world_size > 1 else None
    hidden = [int(x) for x in str(a.hidden_layer_size).split(",") if x.strip()]
    cfg = TaxiDNNConfig(hidden=hidden[0], label=a.target)
    cols = dataset.table_to_numpy(dataset.read_split(os.path.join(a.transformed_data_dir, "train")))
    ids, dense, y = columns_to_tensors(cols, cfg)
    dev = a.device or ("cuda" if torch.cuda.is_available() else "cpu")
    if dev == "cuda" and env.world_size > 1:
        dev = f"cuda:{0 if os.environ.get('MIFX_SHARED_GPU') == '1' else env.local_rank}"
    # shuffled per epoch like the reference's randomised input reader (taxi_utils.py:275-276); same order for any
    # number of ranks (each reads its slice of one global stream)
    tr = TaxiDNNTrainer(TaxiDNN(cfg, seed=0), batch=a.batch_size, lr=a.learning_rate, device=dev, process_group=pg,
                        shuffle_seed=0x5EED)
    tr.set_data(ids, dense, y)
    tr.run(a.steps)  # GPU: hipGraph replays of 50 steps (CPU: eager steps); DP: one all-gather per step
    if env.rank != 0:
        mdist.shutdown()
        return
    ecols = dataset.table_to_numpy(dataset.read_split(os.path.join(a.transformed_data_dir, "eval")))
    eids, edense, ey = columns_to_tensors(ecols, cfg)
    logits = tr.predict_logits(eids, edense)
    acc = float(((logits > 0) == (ey.numpy() > 0.5)).mean())
    export = os.path.join(a.training_output_dir, "export", "export", "1")
    model = tr.model.cpu()
    save_module(export, model, "mifx.models.taxi_dnn:TaxiDNN", {"hidden": cfg.hidden, "seed": None}, None)
    with open(os.path.join(export, "transform_dir.txt"), "w") as f:
        f.write(os.path.abspath(a.transformed_data_dir))
    _metrics(a.training_output_dir, [("accuracy", acc)])
    _write_output(a.training_output_dir_out, a.training_output_dir)
    print(f"trained {a.steps} steps on {dev} x {env.world_size}: eval accuracy {acc:.4f}")
    mdist.shutdown()


def _load_model_and_transform(model_dir: str):
    import torch  # noqa: F401

    from ..models.taxi_dnn import TaxiDNN, TaxiDNNConfig
    from ..serving.saved_model import load
    from ..transform import TransformOutput

    export = os.path.join(model_dir, "export", "export", "1")
    lm = load(export, "cpu")
    with open(os.path.join(export, "transform_dir.txt")) as f:
        tdir = f.read().strip()
    model = lm.model
    assert isinstance(model, TaxiDNN)
    return model, TransformOutput(os.path.join(tdir, "transform_fn")), TaxiDNNConfig


def _score(model, tout, raw_typed: dict):
    import torch

    from ..models.taxi_dnn import columns_to_tensors

    cols = tout.transform_raw_features(raw_typed)
    ids, dense, y = columns_to_tensors(cols, model.cfg)
    with torch.no_grad():
        logits = model(ids, dense).numpy()
    return 1.0 / (1.0 + np.exp(-logits)), (None if y is None else y.numpy())


def tfma(a) -> None:
    """Overall and per-slice accuracy / AUC / loss on the evaluation data."""
    from ..ops.analyzers import auc_from_hist, segment_hist

    with open(a.schema) as f:
        schema = json.load(f)
    model, tout, _ = _load_model_and_transform(a.model)
    raw = _typed(_read_csv(a.evaluation_data, [s["name"] for s in schema]), schema)
    prob, y = _score(model, tout, raw)
    result = {"overall": _slice_metrics(np.zeros(len(prob), np.int64), y, prob, 1, auc_from_hist, segment_hist)[0]}
    for col in [c.strip() for c in a.slice_columns.split(",") if c.strip()]:
        vals = raw[col]
        keys = sorted({str(v) for v in vals}, key=lambda s: (len(s), s))
        seg = np.array([keys.index(str(v)) for v in vals], np.int64)
        per = _slice_metrics(seg, y, prob, len(keys), auc_from_hist, segment_hist)
        result[col] = {k: m for k, m in zip(keys, per)}
    os.makedirs(a.analysis_results_dir, exist_ok=True)
    with open(os.path.join(a.analysis_results_dir, "metrics.json"), "w") as f:
        json.dump(result, f, indent=1)
    _ui(a.analysis_results_dir, [{"type": "table", "format": "csv", "header": ["slice", "value", "count", "accuracy",
                                                                                "auc"],
                                  "source": os.path.join(a.analysis_results_dir, "slices.csv")}])
    with open(os.path.join(a.analysis_results_dir, "slices.csv"), "w") as f:
        for col, per in result.items():
            if col == "overall":
                f.write(f"overall,,{per['count']},{per['accuracy']},{per['auc']}\n")
                continue
            for k, m in per.items():
                f.write(f"{col},{k},{m['count']},{m['accuracy']},{m['auc']}\n")
    _write_output(a.analysis_results_dir_out, a.analysis_results_dir)


def _slice_metrics(seg, y, prob, ns, auc_from_hist, segment_hist):
    sums, hist = segment_hist(seg, y, prob, ns, 1000)
    out = []
    for s in range(ns):
        n = float(sums[s, 0])
        out.append({"count": int(n), "accuracy": float(sums[s, 4] / n) if n else float("nan"),
                    "average_loss": float(sums[s, 3] / n) if n else float("nan"),
                    "auc": auc_from_hist(hist[s])})
    return out


def predict(a) -> None:
    """Batch prediction over a CSV; writes predictions.csv with the target, prediction and probabilities."""
    with open(a.schema) as f:
        schema = json.load(f)
    model, tout, _ = _load_model_and_transform(a.model)
    names = [s["name"] for s in schema]
    raw_str = _read_csv(a.data_file_pattern, names)
    raw = _typed(raw_str, schema)
    probs = []
    n = len(next(iter(raw.values())))
    for s in range(0, n, a.batch_size):  # reference batch-predict B=32
        chunk = {k: v[s:s + a.batch_size] for k, v in raw.items()}
        probs.append(_score(model, tout, chunk)[0])
    prob = np.concatenate(probs) if probs else np.zeros(0)
    os.makedirs(a.predictions_dir, exist_ok=True)
    out = os.path.join(a.predictions_dir, "predictions.csv")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(names + ["target", "predicted", "prob_0", "prob_1"])  # 'target' = the target_column value
        tgt = raw_str.get(a.target_column, np.array([None] * n, dtype=object))
        for i in range(n):
            w.writerow([raw_str[c][i] if raw_str[c][i] is not None else "" for c in names] +
                       ["" if tgt[i] is None else tgt[i], int(prob[i] > 0.5), 1 - prob[i], prob[i]])
    with open(os.path.join(a.predictions_dir, "schema.json"), "w") as f:
        json.dump(schema + [{"name": "target", "type": "NUMBER"}, {"name": "predicted", "type": "NUMBER"}, {"name": "prob_0", "type": "NUMBER"},
                            {"name": "prob_1", "type": "NUMBER"}], f, indent=1)
    _write_output(a.predictions_dir_out, a.predictions_dir)


def _prediction_rows(pred_dir: str, target_column: str):
    with open(os.path.join(pred_dir, "predictions.csv"), newline="") as f:
        rows = list(csv.DictReader(f))
    for r in rows:
        r["target"] = _num(r.get(target_column))
        for k in ("fare", "prob_0", "prob_1", "predicted"):
            if k in r:
                r[k] = _num(r[k])
    return rows


def _num(v):
    try:
        return float(v)
    except (TypeError, ValueError):
        return float("nan")


def confusion_matrix(a) -> None:
    rows = _prediction_rows(a.predictions, a.target_column)
    fn = _compile_target_lambda(a.target_lambda) if a.target_lambda else None
    tgt = [int(bool(fn(r))) if fn else int(r["target"]) for r in rows]
    pred = [int(r["predicted"]) for r in rows]
    labels = [0, 1]
    cm = np.zeros((2, 2), np.int64)
    for t, p in zip(tgt, pred):
        cm[t, p] += 1
    os.makedirs(a.output_dir, exist_ok=True)
    src = os.path.join(a.output_dir, "confusion_matrix.csv")
    with open(src, "w") as f:
        for i in labels:
            for j in labels:
                f.write(f"{i},{j},{cm[i, j]}\n")
    _ui(a.output_dir, [{"type": "confusion_matrix", "format": "csv",
                        "schema": [{"name": "target", "type": "CATEGORY"}, {"name": "predicted", "type": "CATEGORY"},
                                   {"name": "count", "type": "NUMBER"}],
                        "source": src, "labels": [str(x) for x in labels]}])
    acc = float(np.trace(cm) / max(1, cm.sum()))
    _metrics(a.output_dir, [("accuracy-score", acc)])
    _write_output(a.accuracy_out, acc)


def roc(a) -> None:
    rows = _prediction_rows(a.predictions_dir, a.target_column)
    fn = _compile_target_lambda(a.target_lambda) if a.target_lambda else None
    y = np.array([int(fn(r)) if fn else int(r["target"]) for r in rows], np.int64)
    p = np.array([r["prob_1"] for r in rows], np.float64)
    order = np.argsort(-p, kind="stable")
    ys, ps = y[order], p[order]
    tp, fp = np.cumsum(ys), np.cumsum(1 - ys)
    P, N = max(1, ys.sum()), max(1, len(ys) - ys.sum())
    keep = np.r_[np.diff(ps) != 0, True]
    tpr, fpr, thr = np.r_[0, tp[keep] / P], np.r_[0, fp[keep] / N], np.r_[np.inf, ps[keep]]
    auc = float(np.trapezoid(tpr, fpr) if hasattr(np, "trapezoid") else np.trapz(tpr, fpr))
    os.makedirs(a.output_dir, exist_ok=True)
    src = os.path.join(a.output_dir, "roc.csv")
    with open(src, "w") as f:
        for x, t, h in zip(fpr, tpr, thr):
            f.write(f"{x},{t},{h}\n")
    _ui(a.output_dir, [{"type": "roc", "format": "csv",
                        "schema": [{"name": "fpr", "type": "NUMBER"}, {"name": "tpr", "type": "NUMBER"},
                                   {"name": "thresholds", "type": "NUMBER"}], "source": src}])
    _metrics(a.output_dir, [("roc-auc-score", auc)])
    _write_output(a.auc_out, auc)


def deployer(a) -> None:
    """Serving manifests for mifx.serving.server on an AMD GPU node (Deployment + Service)."""
    import yaml

    name = a.server_name
    model_base = os.path.join(a.model_dir, "") if not a.model_dir.endswith("export/export") else a.model_dir
    labels = {"app": name}
    container = {"name": name, "image": a.image,
                 "command": ["python3", "-m", "mifx.serving.server", "--model_name", name, "--model_base_path",
                             model_base, "--rest_api_port", "8500"],
                 "ports": [{"containerPort": 8500}],
                 "resources": {"limits": {"amd.com/gpu": "1"}} if a.gpus else {}}
    pod = {"containers": [container]}
    if a.pvc_name:
        container["volumeMounts"] = [{"name": "model-store", "mountPath": a.mount_path}]
        pod["volumes"] = [{"name": "model-store", "persistentVolumeClaim": {"claimName": a.pvc_name}}]
    deploy = {"apiVersion": "apps/v1", "kind": "Deployment", "metadata": {"name": name, "labels": labels},
              "spec": {"replicas": 1, "selector": {"matchLabels": labels},
                       "template": {"metadata": {"labels": labels}, "spec": pod}}}
    svc = {"apiVersion": "v1", "kind": "Service", "metadata": {"name": name, "labels": labels},
           "spec": {"type": a.service_type, "selector": labels, "ports": [{"name": "rest", "port": 8500,
                                                                            "targetPort": 8500}]}}
    os.makedirs(a.output_dir, exist_ok=True)
    path = os.path.join(a.output_dir, "serving.yaml")
    with open(path, "w") as f:
        yaml.safe_dump_all([deploy, svc], f, sort_keys=False)
    if a.apply:
        from ..kfp.compiler._k8s_helper import K8sHelper

        K8sHelper()._run("apply", "-f", path)
    _write_output(a.manifest_out, path)


def _ui(out_dir: str, outputs: list) -> None:
    with open(os.path.join(out_dir, "mlpipeline-ui-metadata.json"), "w") as f:
        json.dump({"outputs": outputs}, f)
    _write_output(os.environ.get("MIFX_UI_METADATA_PATH"), json.dumps({"outputs": outputs}))


def _metrics(out_dir: str, pairs: list) -> None:
    doc = {"metrics": [{"name": n, "numberValue": float(v), "format": "RAW"} for n, v in pairs]}
    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "mlpipeline-metrics.json"), "w") as f:
        json.dump(doc, f)
    _write_output(os.environ.get("MIFX_METRICS_PATH"), json.dumps(doc))


# ---------------------------------------------------------------------------------------------
# CLI


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="python3 -m mifx.kfp_components.taxi")
    sub = ap.add_subparsers(dest="step", required=True)

    def add(name, fn, args):
        p = sub.add_parser(name)
        for spec in args:
            flag, kw = spec if isinstance(spec, tuple) else (spec, {})
            p.add_argument("--" + flag, **kw)
        p.set_defaults(fn=fn)

    add("tfdv", tfdv, ["inference_data", "validation_data", "column_names", "key_columns", "project",
                       ("mode", {"default": "local"}), "validation_output", "schema_out", "validation_result_out"])
    add("tft", tft, ["training_data_file_pattern", "evaluation_data_file_pattern", "schema", "project",
                     ("mode", {"default": "local"}), "preprocessing_module", "transformed_data_dir",
                     "transformed_data_dir_out"])
    add("dnntrainer", dnntrainer, ["transformed_data_dir", "schema", ("learning_rate", {"type": float, "default": 0.1}),
                                   ("hidden_layer_size", {"default": "1500"}),
                                   ("steps", {"type": int, "default": 3000}), ("target", {"default": "tips"}),
                                   "preprocessing_module", "training_output_dir",
                                   ("batch_size", {"type": int, "default": 32}), "device", "training_output_dir_out",
                                   ("num_gpus", {"type": int, "default": 1})])
    add("tfma", tfma, ["model", "evaluation_data", "schema", "project", ("mode", {"default": "local"}),
                       ("slice_columns", {"default": ""}), "analysis_results_dir", "analysis_results_dir_out"])
    add("predict", predict, ["data_file_pattern", "schema", ("target_column", {"default": "tips"}), "model",
                             ("mode", {"default": "local"}), "project", "predictions_dir",
                             ("batch_size", {"type": int, "default": 32}), "predictions_dir_out"])
    add("confusion_matrix", confusion_matrix, ["predictions", ("target_lambda", {"default": ""}),
                                               ("target_column", {"default": "target"}), "output_dir",
                                               "accuracy_out"])
    add("roc", roc, ["predictions_dir", ("target_lambda", {"default": ""}), ("target_column", {"default": "target"}),
                     "output_dir", "auc_out"])
    add("deployer", deployer, ["model_dir", "server_name", "cluster_name", "pvc_name",
                               ("service_type", {"default": "ClusterIP"}), ("image", {"default": "mifx/mifx-rocm:latest"}),
                               ("mount_path", {"default": "/mnt"}), ("gpus", {"type": int, "default": 1}),
                               ("apply", {"type": int, "default": 0}), "output_dir", "manifest_out"])
    return ap


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = build_parser().parse_args(argv)
    a._argv = argv
    a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
