"""Schema inference and statistics validation (TFDV semantics).

Reference: `02_TensorFlow_Data_Validation.ipynb` cells 13-34 — `infer_schema`, `validate_statistics`
(missing/new columns, unexpected string values vs `min_domain_mass`, presence, type), environments
(`TRAINING`/`SERVING`, `not_in_environment` for the label), and train-vs-serving skew /
span-to-span drift with L-infinity comparators (thresholds 0.01 / 0.001 in the notebook).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field

import numpy as np

from .schema import Feature, IntDomain, Schema, StringDomain
from .stats import get_dataset

_TYPE = {"INT": "INT", "FLOAT": "FLOAT", "STRING": "BYTES"}


def infer_schema(stats: dict, infer_feature_shape: bool = True, max_string_domain_size: int = 100) -> Schema:
    ds = stats["datasets"][0]
    n = ds["num_examples"]
    schema = Schema()
    for f in ds["features"]:
        st = f.get("num_stats") or f.get("string_stats")
        c = st["common_stats"]
        feat = Feature(name=f["name"], type=_TYPE[f["type"]])
        if c["num_missing"] == 0 and n > 0:
            feat.presence_min_fraction = 1.0
            feat.presence_min_count = 1
            if infer_feature_shape:
                feat.univalent_shape = True
        else:
            feat.presence_min_count = 1
            feat.value_count_min, feat.value_count_max = 1, 1
        if f["type"] == "STRING":
            vc = st.get("value_counts", {})
            if 0 < len(vc) <= max_string_domain_size:
                schema.string_domain.append(StringDomain(f["name"], sorted(vc)))
                feat.domain = f["name"]
        schema.feature.append(feat)
    return schema


@dataclass
class Anomalies:
    anomaly_info: dict = field(default_factory=dict)

    def add(self, feature: str, kind: str, short: str, desc: str) -> None:
        e = self.anomaly_info.setdefault(feature, {"severity": "ERROR", "reason": []})
        e["reason"].append({"type": kind, "short_description": short, "description": desc})
        e["short_description"] = e["reason"][0]["short_description"] if len(e["reason"]) == 1 else "Multiple errors"
        e["description"] = " ".join(r["description"] for r in e["reason"])

    def __bool__(self):
        return bool(self.anomaly_info)

    def to_json(self) -> str:
        return json.dumps({"anomaly_info": self.anomaly_info}, indent=1)

    @staticmethod
    def from_json(s: str) -> "Anomalies":
        return Anomalies(json.loads(s).get("anomaly_info", {}))

    def frame(self):
        import pandas as pd

        rows = [{"Feature name": k, "Anomaly short description": v["short_description"],
                 "Anomaly long description": v["description"]} for k, v in sorted(self.anomaly_info.items())]
        return pd.DataFrame(rows)


def display_anomalies(anomalies: Anomalies) -> str:
    if not anomalies:
        return "No anomalies found."
    return anomalies.frame().to_string(index=False)


def _in_env(f: Feature, env: str | None, schema: Schema) -> bool:
    if env is None:
        return True
    if env in f.not_in_environment:
        return False
    if f.in_environment:
        return env in f.in_environment
    return not schema.default_environment or env in schema.default_environment


def _dist(fs: dict) -> dict:
    st = fs.get("string_stats") or fs.get("num_stats") or {}
    vc = st.get("value_counts") or {}
    tot = float(sum(vc.values())) or 1.0
    return {k: v / tot for k, v in vc.items()}


def linf_distance(a: dict, b: dict) -> tuple[float, str]:
    pa_, pb = _dist(a), _dist(b)
    best, arg = 0.0, ""
    for k in set(pa_) | set(pb):
        d = abs(pa_.get(k, 0.0) - pb.get(k, 0.0))
        if d > best:
            best, arg = d, k
    return best, arg


def validate_statistics(statistics: dict, schema: Schema, environment: str | None = None,
                        previous_statistics: dict | None = None, serving_statistics: dict | None = None) -> Anomalies:
    ds = get_dataset(statistics)
    n = ds["num_examples"]
    feats = {f["name"]: f for f in ds["features"]}
    an = Anomalies()
    for name, fs in feats.items():
        try:
            sf = schema.get_feature(name)
        except KeyError:
            an.add(name, "SCHEMA_NEW_COLUMN", "New column", "New column (column in data but not in schema)")
            continue
        if not _in_env(sf, environment, schema):
            continue
        st = fs.get("num_stats") or fs.get("string_stats")
        present = st["common_stats"]["num_non_missing"]
        if _TYPE[fs["type"]] != sf.type and not (sf.type == "FLOAT" and fs["type"] == "INT"):
            an.add(name, "UNEXPECTED_DATA_TYPE", "Unexpected data type",
                   f"Expected data of type: {sf.type} but got {_TYPE[fs['type']]}")
        if sf.presence_min_fraction is not None and n and present / n < sf.presence_min_fraction:
            an.add(name, "FEATURE_TYPE_LOW_FRACTION_PRESENT", "Column dropped",
                   f"The feature was present in fewer examples than expected: minimum fraction = "
                   f"{sf.presence_min_fraction}, actual = {present / n:.4g}")
        if sf.presence_min_count is not None and present < sf.presence_min_count:
            an.add(name, "FEATURE_TYPE_LOW_NUMBER_PRESENT", "Column dropped",
                   f"The feature was present in fewer examples than expected: minimum count = "
                   f"{sf.presence_min_count}, actual = {present}")
        dom = schema.get_domain(sf)
        if isinstance(dom, StringDomain) and "string_stats" in fs:
            vc = fs["string_stats"].get("value_counts", {})
            allowed = set(dom.value)
            bad = {k: v for k, v in vc.items() if k not in allowed}
            mass = sum(bad.values()) / max(1, sum(vc.values()))
            min_mass = sf.min_domain_mass if sf.min_domain_mass is not None else 1.0
            if bad and mass > 1.0 - min_mass + 1e-12:
                ex = ", ".join(sorted(bad)[:10])
                an.add(name, "ENUM_TYPE_UNEXPECTED_STRING_VALUES", "Unexpected string values",
                       f"Examples contain values missing from the schema: {ex} (~{100 * mass:.0f}% of the examples)")
        elif isinstance(dom, IntDomain) and "num_stats" in fs and present:
            ns = fs["num_stats"]
            if dom.min is not None and ns["min"] < dom.min:
                an.add(name, "INT_TYPE_SMALL_INT", "Out-of-range values",
                       f"Unexpectedly small value: {ns['min']} < {dom.min}")
            if dom.max is not None and ns["max"] > dom.max:
                an.add(name, "INT_TYPE_BIG_INT", "Out-of-range values",
                       f"Unexpectedly large value: {ns['max']} > {dom.max}")
    for sf in schema.feature:
        if sf.name in feats or not _in_env(sf, environment, schema):
            continue
        if (sf.presence_min_count or 0) >= 1 or (sf.presence_min_fraction or 0) > 0:
            an.add(sf.name, "SCHEMA_MISSING_COLUMN", "Column dropped", "Column is completely missing")
    for other, attr, label in ((serving_statistics, "skew_linf_threshold", "skew"),
                               (previous_statistics, "drift_linf_threshold", "drift")):
        if other is None:
            continue
        ofeats = {f["name"]: f for f in get_dataset(other)["features"]}
        for sf in schema.feature:
            th = getattr(sf, attr)
            if th is None or sf.name not in feats or sf.name not in ofeats:
                continue
            d, arg = linf_distance(feats[sf.name], ofeats[sf.name])
            if d > th:
                kind = "COMPARATOR_L_INFTY_HIGH"
                an.add(sf.name, kind, f"High Linfty distance between {'training and serving' if label == 'skew' else 'current and previous'}",
                       f"The Linfty distance between {label} inputs is {d:.4g} (up to six significant digits), "
                       f"above the threshold {th}. The feature value with maximum difference is: {arg}")
    return an


def set_domain(schema: Schema, feature: str, domain) -> None:
    f = schema.get_feature(feature)
    if isinstance(domain, StringDomain):
        schema.string_domain = [d for d in schema.string_domain if d.name != domain.name] + [domain]
        f.domain, f.int_domain, f.float_domain = domain.name, None, None
    elif isinstance(domain, IntDomain):
        f.int_domain, f.domain = domain, None
    else:
        f.float_domain, f.domain = domain, None


def summarize_l_inf(stats_a: dict, stats_b: dict) -> dict:
    """Per-feature L-infinity distances (categorical features) between two statistics sets."""
    fa = {f["name"]: f for f in get_dataset(stats_a)["features"]}
    fb = {f["name"]: f for f in get_dataset(stats_b)["features"]}
    return {k: linf_distance(fa[k], fb[k])[0] for k in fa if k in fb and _dist(fa[k]) and _dist(fb[k])}


_ = np  # numpy used by callers via stats arrays
