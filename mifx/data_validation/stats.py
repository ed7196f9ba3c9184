"""Dataset statistics (TFDV `DatasetFeatureStatisticsList` semantics, JSON encoded).

Reference: `02_TensorFlow_Data_Validation.ipynb` cells 9-15 (generate_statistics_from_csv,
visualize, compare train vs eval) and SURVEY KN11 (per-feature count/missing/mean/std/min/max/
zeros/quantile + equal-width histograms, unique count, top-k strings). Numeric columns reduce on
the GPU through mifx.ops.analyzers when a device is given; otherwise numpy.
"""
from __future__ import annotations

import json
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.csv as pacsv

NUM_HIST_BUCKETS = 10
NUM_QUANTILE_BUCKETS = 10
TOP_K = 20


def _common(n: int, present: int) -> dict:
    return {"num_non_missing": int(present), "num_missing": int(n - present), "min_num_values": 1 if present else 0,
            "max_num_values": 1 if present else 0, "avg_num_values": 1.0 if present else 0.0,
            "tot_num_values": int(present)}


def _gpu(device) -> bool:
    return device is not None and str(device).startswith("cuda")


def _num_stats(vals: np.ndarray, n: int, device=None) -> dict:
    """On a GPU the column goes to the device ONCE and every statistic is a kernel there: moments (fp64 Welford),
    the equal-width histogram (hist_k with np.histogram's edges), quantiles + median (exact order statistics by
    histogram narrowing) -- bit-identical to the numpy path (tests/test_analyzers_quantiles.py)."""
    from ..ops import analyzers

    present = vals.size
    st = {"common_stats": _common(n, present)}
    if present == 0:
        return st
    x = vals.astype(np.float64)
    if _gpu(device):
        import torch

        x = torch.from_numpy(np.ascontiguousarray(x)).to(device)
        mom = analyzers.column_moments(x, device=device)
    else:
        mom = {"mean": float(x.mean()), "std": float(x.std()), "min": float(x.min()), "max": float(x.max()),
               "zeros": int((x == 0).sum())}
    dev = device if _gpu(device) else None
    lo, hi = mom["min"], mom["max"]
    edges = np.linspace(lo, hi, NUM_HIST_BUCKETS + 1) if hi > lo else np.array([lo, hi])
    counts = analyzers.histogram(x, edges, device=dev)
    qgrid = np.linspace(0, 1, NUM_QUANTILE_BUCKETS + 1)
    qv = analyzers.quantiles(x, np.concatenate([qgrid, [0.5]]), method="linear", device=dev)
    qs, median = qv[:-1], float(qv[-1])
    st.update(mean=mom["mean"], std_dev=mom["std"], num_zeros=mom["zeros"], min=lo, max=hi,
              median=median,
              histograms=[
                  {"type": "STANDARD", "num_nan": 0, "buckets": [
                      {"low_value": float(edges[i]), "high_value": float(edges[i + 1]), "sample_count": float(c)}
                      for i, c in enumerate(counts)]},
                  {"type": "QUANTILES", "buckets": [
                      {"low_value": float(qs[i]), "high_value": float(qs[i + 1]),
                       "sample_count": float(present) / NUM_QUANTILE_BUCKETS} for i in range(NUM_QUANTILE_BUCKETS)]}])
    return st


def _string_stats(vals, n: int, device=None) -> dict:
    """vals: object array of str, or (GPU) the Arrow column itself -- the device hash-table count
    (csrc/vocab.hip, exact with collision fallback) reads its buffers without a per-row Python pass."""
    size = len(vals)
    st = {"common_stats": _common(n, size)}
    if size == 0:
        return st
    if _gpu(device) and not isinstance(vals, np.ndarray):
        import pyarrow.compute as pc

        from ..ops import vocab as V

        got = V.count_unique(vals, device=device) or V.count_unique(vals, device=None)
        vc = pd.Series(got[1], index=got[0], dtype=np.int64)
        avg_len = float(pc.mean(pc.utf8_length(vals)).as_py())
    else:
        s = pd.Series(np.asarray(vals, dtype=object).astype(str))
        vc = s.value_counts()
        avg_len = float(s.str.len().mean())
    vc = vc.sort_index(kind="stable").sort_values(ascending=False, kind="stable")
    st.update(unique=int(vc.size), avg_length=avg_len,
              top_values=[{"value": str(k), "frequency": float(v)} for k, v in vc.head(TOP_K).items()],
              rank_histogram={"buckets": [{"low_rank": i, "high_rank": i, "label": str(k), "sample_count": float(v)}
                                          for i, (k, v) in enumerate(vc.head(50).items())]},
              value_counts={str(k): int(v) for k, v in vc.items()})
    return st


def _column(col: pa.ChunkedArray, device=None):
    col = col.combine_chunks() if isinstance(col, pa.ChunkedArray) else col
    valid = col.drop_null()
    if pa.types.is_string(col.type) or pa.types.is_large_string(col.type) or pa.types.is_binary(col.type):
        if _gpu(device):
            return "STRING", valid
        return "STRING", np.array(valid.to_pylist(), dtype=object)
    if pa.types.is_integer(col.type) or pa.types.is_boolean(col.type):
        return "INT", valid.to_numpy(zero_copy_only=False).astype(np.int64)
    if pa.types.is_floating(col.type):
        v = valid.to_numpy(zero_copy_only=False).astype(np.float64)
        return "FLOAT", v[~np.isnan(v)]
    if pa.types.is_null(col.type):
        return "STRING", np.array([], dtype=object)
    raise TypeError(f"unsupported column type {col.type}")


def generate_statistics_from_table(table: pa.Table, name: str = "", device=None) -> dict:
    n = table.num_rows
    feats = []
    for cname in table.column_names:
        kind, vals = _column(table.column(cname), device)
        f = {"name": cname, "type": kind}
        if kind == "STRING":
            f["string_stats"] = _string_stats(vals, n, device)
        else:
            f["num_stats"] = _num_stats(vals, n, device)
            if kind == "INT":  # categorical view for skew/drift comparators on int features
                from ..ops.analyzers import int_value_counts

                u, c = int_value_counts(vals, device=device if _gpu(device) else None)
                if u.size <= 10000:
                    f["num_stats"]["value_counts"] = {str(int(a)): int(b) for a, b in zip(u, c)}
        feats.append(f)
    return {"datasets": [{"name": name, "num_examples": int(n), "features": feats}]}


_CSV_CONVERT = pacsv.ConvertOptions(strings_can_be_null=True)  # empty CSV field == missing (TFDV semantics)


def read_csv_table(path: str) -> pa.Table:
    if os.path.isdir(path):
        files = sorted(os.path.join(path, f) for f in os.listdir(path) if f.endswith(".csv"))
        return pa.concat_tables([pacsv.read_csv(f, convert_options=_CSV_CONVERT) for f in files],
                                promote_options="default")
    return pacsv.read_csv(path, convert_options=_CSV_CONVERT)


def generate_statistics_from_csv(path: str, name: str = "", device=None) -> dict:
    return generate_statistics_from_table(read_csv_table(path), name=name, device=device)


def generate_statistics_from_dataframe(df: pd.DataFrame, name: str = "") -> dict:
    return generate_statistics_from_table(pa.Table.from_pandas(df, preserve_index=False), name=name)


def merge_statistics(stats_list: list[dict]) -> dict:
    return {"datasets": [d for s in stats_list for d in s["datasets"]]}


def write_stats(stats: dict, path: str) -> None:
    with open(path, "w") as f:
        json.dump(stats, f)


def load_statistics(path: str) -> dict:
    if os.path.isdir(path):
        path = os.path.join(path, "stats.json")
    with open(path) as f:
        return json.load(f)


def get_dataset(stats: dict, name: str | None = None) -> dict:
    for d in stats["datasets"]:
        if name is None or d["name"] == name:
            return d
    raise KeyError(f"dataset {name} not in statistics")


def get_feature_stats(stats: dict, feature: str, dataset: str | None = None) -> dict:
    for f in get_dataset(stats, dataset)["features"]:
        if f["name"] == feature:
            return f
    raise KeyError(feature)


def stats_frame(stats: dict, dataset: str | None = None) -> pd.DataFrame:
    """Tabular summary (the numbers `tfdv.visualize_statistics` renders)."""
    rows = []
    for f in get_dataset(stats, dataset)["features"]:
        s = f.get("num_stats") or f.get("string_stats")
        c = s["common_stats"]
        row = {"feature": f["name"], "type": f["type"], "count": c["num_non_missing"],
               "missing": c["num_missing"]}
        if "num_stats" in f:
            row.update({k: s.get(k) for k in ("mean", "std_dev", "num_zeros", "min", "median", "max")})
        else:
            row.update(unique=s.get("unique"), top=(s.get("top_values") or [{}])[0].get("value"),
                       avg_length=s.get("avg_length"))
        rows.append(row)
    return pd.DataFrame(rows).set_index("feature")


def visualize_statistics(stats: dict, rhs: dict | None = None, lhs_name: str = "lhs", rhs_name: str = "rhs") -> str:
    """Text rendering of one or two statistics sets (side by side)."""
    a = stats_frame(stats)
    if rhs is None:
        return a.to_string()
    b = stats_frame(rhs)
    return pd.concat([a, b], axis=1, keys=[lhs_name, rhs_name]).to_string()
