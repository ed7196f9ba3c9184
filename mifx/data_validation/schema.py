"""Schema model compatible with TF Metadata `schema.pbtxt` text format.

Reference workflow: `02_TensorFlow_Data_Validation.ipynb` (infer_schema, relax domains with
`min_domain_mass=0.9`, add a domain value, environments TRAINING/SERVING with
`not_in_environment`, skew/drift L-infinity comparators, freeze `schema.pbtxt`) and
`06_Airflow_Feature_Analysis.ipynb` (read the SchemaGen artifact's `schema.pbtxt`).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Any

# --------------------------------------------------------------------------- text format
_TOKEN = re.compile(r'\s*(?:(#[^\n]*)|("(?:[^"\\]|\\.)*")|(\'(?:[^\'\\]|\\.)*\')|([{}:\[\],])|([^\s{}:\[\],"\']+))')


def _tokens(text: str):
    pos = 0
    while pos < len(text):
        m = _TOKEN.match(text, pos)
        if not m or m.end() == pos:
            if text[pos:].strip() == "":
                return
            raise ValueError(f"bad pbtxt near {text[pos:pos + 30]!r}")
        pos = m.end()
        if m.group(1):
            continue
        if m.group(2) or m.group(3):
            s = (m.group(2) or m.group(3))[1:-1]
            yield ("str", bytes(s, "utf-8").decode("unicode_escape"))
        elif m.group(4):
            yield ("sym", m.group(4))
        elif m.group(5):
            yield ("atom", m.group(5))


def parse_pbtxt(text: str) -> dict[str, list]:
    toks = list(_tokens(text))
    i = 0

    def value(tok):
        kind, v = tok
        if kind == "str":
            return v
        if v in ("true", "True"):
            return True
        if v in ("false", "False"):
            return False
        try:
            return int(v)
        except ValueError:
            try:
                return float(v)
            except ValueError:
                return v  # enum identifier

    def block(end: str | None):
        nonlocal i
        out: dict[str, list] = {}
        while i < len(toks):
            kind, v = toks[i]
            if kind == "sym" and v == end:
                i += 1
                return out
            name = v
            i += 1
            if toks[i] == ("sym", ":"):
                i += 1
            if toks[i] == ("sym", "{"):
                i += 1
                out.setdefault(name, []).append(block("}"))
            elif toks[i] == ("sym", "["):
                i += 1
                while toks[i] != ("sym", "]"):
                    if toks[i] != ("sym", ","):
                        out.setdefault(name, []).append(value(toks[i]))
                    i += 1
                i += 1
            else:
                out.setdefault(name, []).append(value(toks[i]))
                i += 1
        return out

    return block(None)


def _fmt(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"') + '"'
    if isinstance(v, float):
        return repr(v)
    return str(v)


class Enum(str):
    """marks a string written without quotes (protobuf enum value)."""


def dump_pbtxt(d: dict, indent: int = 0) -> str:
    pad = "  " * indent
    lines = []
    for k, vals in d.items():
        for v in (vals if isinstance(vals, list) else [vals]):
            if v is None:
                continue
            if isinstance(v, dict):
                lines.append(f"{pad}{k} {{")
                lines.append(dump_pbtxt(v, indent + 1))
                lines.append(f"{pad}}}")
            elif isinstance(v, Enum):
                lines.append(f"{pad}{k}: {v}")
            else:
                lines.append(f"{pad}{k}: {_fmt(v)}")
    return "\n".join(x for x in lines if x != "")


# ------------------------------------------------------------------------------ model
@dataclass
class StringDomain:
    name: str
    value: list[str] = field(default_factory=list)


@dataclass
class IntDomain:
    min: int | None = None
    max: int | None = None
    is_categorical: bool = False


@dataclass
class FloatDomain:
    min: float | None = None
    max: float | None = None


@dataclass
class Feature:
    name: str
    type: str = "BYTES"  # INT | FLOAT | BYTES
    domain: str | None = None  # name of a top-level string_domain
    int_domain: IntDomain | None = None
    float_domain: FloatDomain | None = None
    presence_min_fraction: float | None = None
    presence_min_count: int | None = None
    value_count_min: int | None = None
    value_count_max: int | None = None
    univalent_shape: bool = False
    min_domain_mass: float | None = None  # distribution_constraints
    skew_linf_threshold: float | None = None
    drift_linf_threshold: float | None = None
    in_environment: list[str] = field(default_factory=list)
    not_in_environment: list[str] = field(default_factory=list)

    def to_dict(self) -> dict:
        d: dict[str, Any] = {"name": self.name}
        if self.value_count_min is not None or self.value_count_max is not None:
            vc = {}
            if self.value_count_min is not None:
                vc["min"] = self.value_count_min
            if self.value_count_max is not None:
                vc["max"] = self.value_count_max
            d["value_count"] = vc
        d["type"] = Enum(self.type)
        if self.domain:
            d["domain"] = self.domain
        if self.int_domain:
            idm = {k: v for k, v in (("min", self.int_domain.min), ("max", self.int_domain.max)) if v is not None}
            if self.int_domain.is_categorical:
                idm["is_categorical"] = True
            d["int_domain"] = idm
        if self.float_domain:
            d["float_domain"] = {k: v for k, v in (("min", self.float_domain.min), ("max", self.float_domain.max))
                                 if v is not None}
        if self.presence_min_fraction is not None or self.presence_min_count is not None:
            pr = {}
            if self.presence_min_fraction is not None:
                pr["min_fraction"] = float(self.presence_min_fraction)
            if self.presence_min_count is not None:
                pr["min_count"] = int(self.presence_min_count)
            d["presence"] = pr
        if self.univalent_shape:
            d["shape"] = {"dim": {"size": 1}}
        if self.min_domain_mass is not None:
            d["distribution_constraints"] = {"min_domain_mass": float(self.min_domain_mass)}
        if self.skew_linf_threshold is not None:
            d["skew_comparator"] = {"infinity_norm": {"threshold": float(self.skew_linf_threshold)}}
        if self.drift_linf_threshold is not None:
            d["drift_comparator"] = {"infinity_norm": {"threshold": float(self.drift_linf_threshold)}}
        if self.in_environment:
            d["in_environment"] = list(self.in_environment)
        if self.not_in_environment:
            d["not_in_environment"] = list(self.not_in_environment)
        return d

    @staticmethod
    def from_dict(d: dict) -> "Feature":
        g = lambda k: d.get(k, [None])[0]  # noqa: E731
        f = Feature(name=g("name"), type=str(g("type") or "BYTES"))
        f.domain = g("domain")
        if "int_domain" in d:
            x = d["int_domain"][0]
            f.int_domain = IntDomain(x.get("min", [None])[0], x.get("max", [None])[0],
                                     bool(x.get("is_categorical", [False])[0]))
        if "float_domain" in d:
            x = d["float_domain"][0]
            f.float_domain = FloatDomain(x.get("min", [None])[0], x.get("max", [None])[0])
        if "presence" in d:
            x = d["presence"][0]
            f.presence_min_fraction = x.get("min_fraction", [None])[0]
            f.presence_min_count = x.get("min_count", [None])[0]
        if "value_count" in d:
            x = d["value_count"][0]
            f.value_count_min = x.get("min", [None])[0]
            f.value_count_max = x.get("max", [None])[0]
        f.univalent_shape = "shape" in d
        if "distribution_constraints" in d:
            f.min_domain_mass = d["distribution_constraints"][0].get("min_domain_mass", [1.0])[0]
        for comp in ("skew", "drift"):
            if f"{comp}_comparator" in d:
                th = d[f"{comp}_comparator"][0].get("infinity_norm", [{}])[0].get("threshold", [None])[0]
                setattr(f, f"{comp}_linf_threshold", th)
        f.in_environment = list(d.get("in_environment", []))
        f.not_in_environment = list(d.get("not_in_environment", []))
        return f


@dataclass
class Schema:
    feature: list[Feature] = field(default_factory=list)
    string_domain: list[StringDomain] = field(default_factory=list)
    default_environment: list[str] = field(default_factory=list)

    def get_feature(self, name: str) -> Feature:
        for f in self.feature:
            if f.name == name:
                return f
        raise KeyError(f"feature {name} not in schema")

    def get_domain(self, name_or_feature) -> StringDomain | IntDomain | FloatDomain | None:
        f = name_or_feature if isinstance(name_or_feature, Feature) else self.get_feature(name_or_feature)
        if f.domain:
            for d in self.string_domain:
                if d.name == f.domain:
                    return d
        return f.int_domain or f.float_domain

    def feature_names(self) -> list[str]:
        return [f.name for f in self.feature]

    def to_pbtxt(self) -> str:
        d = {"feature": [f.to_dict() for f in self.feature],
             "string_domain": [{"name": s.name, "value": list(s.value)} for s in self.string_domain]}
        if self.default_environment:
            d["default_environment"] = list(self.default_environment)
        return dump_pbtxt(d) + "\n"

    @staticmethod
    def from_pbtxt(text: str) -> "Schema":
        d = parse_pbtxt(text)
        return Schema(feature=[Feature.from_dict(x) for x in d.get("feature", [])],
                      string_domain=[StringDomain(x["name"][0], list(x.get("value", [])))
                                     for x in d.get("string_domain", [])],
                      default_environment=list(d.get("default_environment", [])))

    # tft-style feature spec: name -> (dtype, fixed_len | var_len)
    def as_feature_spec(self) -> dict[str, dict]:
        out = {}
        for f in self.feature:
            dtype = {"INT": "int64", "FLOAT": "float32", "BYTES": "string"}[f.type]
            fixed = f.univalent_shape and (f.presence_min_fraction or 0) >= 1.0
            out[f.name] = {"dtype": dtype, "kind": "fixed_len" if fixed else "var_len"}
        return out


def write_schema_text(schema: Schema, path: str) -> None:
    with open(path, "w") as f:
        f.write(schema.to_pbtxt())


def load_schema_text(path: str) -> Schema:
    with open(path) as f:
        return Schema.from_pbtxt(f.read())
