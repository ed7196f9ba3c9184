"""Full-pass analyzers + per-row mappers (tf.Transform-equivalent) with analyze/apply phases.

Reference semantics (`airflow-dags/taxi_utils.py:86-145`, `kubeflow-pipelines/taxi/preprocessing.py:65-101`,
`03_TensorFlow_Transform.ipynb`): `scale_to_z_score`, `compute_and_apply_vocabulary(top_k,
num_oov_buckets)`, `bucketize(x, num_buckets)` (quantile boundaries), `scale_to_0_1`, `mean`,
`string_to_int`, `_fill_in_missing`. A user `preprocessing_fn(inputs) -> outputs` runs twice:

* ANALYZE (Transform component, full dataset): each analyzer computes its statistics over the whole
  column and records them, in call order, into a :class:`TransformState`;
* APPLY (transformed examples, eval and serving): the same function replays with the recorded
  constants — identical math on any batch, so train/serve skew cannot creep in.

Numeric analyzers reduce on the GPU (mifx.ops.analyzers HIP kernels) when a device is set.

Parity notes: vocabulary order is frequency-descending with ties broken by value descending
(tft's ordering); OOV buckets use a stable 64-bit FNV-1a hash instead of TF's FarmHash (bucket
ids of OOV strings are therefore not byte-identical to TF — parity unpinned, no TF available).
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
from dataclasses import dataclass, field
from typing import Any

import numpy as np

_LOCAL = threading.local()


@dataclass
class TransformState:
    entries: list = field(default_factory=list)  # [{"kind":..., "params":..., "values":...}]

    def to_json(self) -> str:
        return json.dumps({"entries": self.entries})

    @staticmethod
    def from_json(s: str) -> "TransformState":
        return TransformState(json.loads(s)["entries"])


class _Ctx:
    def __init__(self, mode: str, state: TransformState, device=None):
        self.mode = mode
        self.state = state
        self.cursor = 0
        self.device = device


def _ctx() -> _Ctx:
    c = getattr(_LOCAL, "ctx", None)
    if c is None:
        raise RuntimeError("mifx.transform analyzers must run inside analyze()/apply()")
    return c


@contextlib.contextmanager
def _phase(mode: str, state: TransformState, device=None):
    prev = getattr(_LOCAL, "ctx", None)
    _LOCAL.ctx = _Ctx(mode, state, device)
    try:
        yield _LOCAL.ctx
    finally:
        _LOCAL.ctx = prev


class ShardStop(Exception):
    """Raised in the SHARD phase (mifx.transform.parallel) at the analyzer being accumulated: carries its kind,
    parameters and this shard's input to it; the rest of preprocessing_fn is not run."""

    def __init__(self, kind: str, params: dict, data):
        super().__init__(kind)
        self.kind, self.params, self.data = kind, params, data


def _analyzer(kind: str, params: dict, compute, data=None):
    """One full-pass analyzer call. `data`: its input (the column; the row count for size), which the sharded
    analyze (mifx.transform.parallel) accumulates per shard and merges instead of calling `compute`."""
    c = _ctx()
    if c.mode == "shard":  # analyzers before the target replay their merged values; the target stops the fn
        if c.cursor < len(c.state.entries):
            e = c.state.entries[c.cursor]
            c.cursor += 1
            if e["kind"] != kind:
                raise RuntimeError(f"analyzer order changed: recorded {e['kind']}, now {kind}")
            return e["values"]
        raise ShardStop(kind, params, data)
    if c.mode == "analyze":
        values = compute()
        c.state.entries.append({"kind": kind, "params": params, "values": values})
        return values
    if c.cursor >= len(c.state.entries):
        raise RuntimeError("preprocessing_fn called more analyzers than were recorded")
    e = c.state.entries[c.cursor]
    c.cursor += 1
    if e["kind"] != kind:
        raise RuntimeError(f"analyzer order changed: recorded {e['kind']}, now {kind}")
    return e["values"]


def analyze(preprocessing_fn, inputs: dict, device=None) -> tuple[dict, TransformState]:
    """Run the ANALYZE phase over the full dataset; returns (transformed columns, state)."""
    st = TransformState()
    with _phase("analyze", st, device):
        out = preprocessing_fn(dict(inputs))
    return _materialize(out), st


def apply(preprocessing_fn, inputs: dict, state: TransformState, device=None) -> dict:
    """APPLY phase: replay with recorded analyzer constants (mappers run on `device` when set)."""
    with _phase("apply", state, device):
        out = preprocessing_fn(dict(inputs))
    return _materialize(out)


def _materialize(out: dict) -> dict:
    return {k: np.asarray(_np(v)) for k, v in out.items()}


# ------------------------------------------------------------------------------- helpers
def _is_arrow(x) -> bool:
    """A pyarrow (Chunked)Array: string columns may stay in Arrow form (offsets + bytes buffers) so the
    GPU vocabulary kernels read them without a per-row Python pass."""
    mod = type(x).__module__
    return mod.startswith("pyarrow")


def _arrow_is_str(x) -> bool:
    import pyarrow as pa

    return pa.types.is_string(x.type) or pa.types.is_large_string(x.type) or pa.types.is_binary(x.type) \
        or pa.types.is_large_binary(x.type)


def _np(x):
    return np.array(x.to_pylist(), dtype=object) if _is_arrow(x) else x


def _num(x) -> np.ndarray:
    """Numeric column as float64, missing -> NaN (Arrow columns converted without a per-row Python pass)."""
    if _is_arrow(x):
        import pyarrow as pa

        a = x.combine_chunks() if isinstance(x, pa.ChunkedArray) else x
        if pa.types.is_integer(a.type) or pa.types.is_floating(a.type) or pa.types.is_boolean(a.type):
            return a.cast(pa.float64()).to_numpy(zero_copy_only=False)
        x = _np(x)
    a = np.asarray(x)
    if a.dtype == object:
        import pandas as pd

        a = pd.to_numeric(pd.Series(a, dtype=object), errors="coerce").to_numpy(dtype=np.float64, na_value=np.nan)
    return a.astype(np.float64)


def to_float(x) -> np.ndarray:
    """Public: a column as float64 with missing values as NaN (e.g. the taxi label rule's NaN fare test)."""
    return _num(x)


def _str(x) -> np.ndarray:
    a = np.asarray(_np(x), dtype=object)
    return np.array(["" if v is None else (v.decode() if isinstance(v, bytes) else str(v)) for v in a], dtype=object)


def _str_or_arrow(x):
    """Arrow string columns pass through untouched (GPU paths consume their buffers); else _str."""
    return x if _is_arrow(x) and _arrow_is_str(x) else _str(x)


def fill_in_missing(x, default=None) -> np.ndarray:
    """Densify an optional column (`taxi_utils.py:86-103`): None/NaN -> '' or 0."""
    if _is_arrow(x):
        if _arrow_is_str(x):
            import pyarrow.compute as pc

            return pc.fill_null(x, "" if default is None else default) if x.null_count else x
        x = _np(x)
    a = np.asarray(x, dtype=object) if not isinstance(x, np.ndarray) else x
    if a.dtype == object:  # vectorised: pandas missing mask + dtype inference, no per-row Python loop
        import pandas as pd

        ser = pd.Series(a, dtype=object)
        miss = ser.isna().to_numpy()
        kind = pd.api.types.infer_dtype(ser[~miss], skipna=True) if (~miss).any() else "empty"
        # any column holding a str / bytes value stays a string column ("mixed-integer": ints mixed with strings)
        is_str = kind in ("string", "bytes", "mixed", "mixed-integer", "mixed-integer-float")
        d = ("" if is_str else 0) if default is None else default
        if is_str:
            out = a.copy()
            out[miss] = d
            return out
        out = pd.to_numeric(ser, errors="coerce").to_numpy(dtype=np.float64, na_value=np.nan)
        out[miss] = d
        if np.all(np.mod(out, 1) == 0):
            out = out.astype(np.int64)
        return out
    if np.issubdtype(a.dtype, np.floating):
        return np.where(np.isnan(a), 0.0 if default is None else default, a)
    return a


GPU_MIN_ROWS = int(os.environ.get("MIFX_GPU_ANALYZER_MIN_ROWS", "8192"))


def _gpu_ctx(n: int):
    """The active phase's device when it is a GPU and the column is big enough to be worth a launch."""
    c = getattr(_LOCAL, "ctx", None)
    if c is None or c.device is None or n < GPU_MIN_ROWS:
        return None
    import torch

    return c.device if torch.device(c.device).type == "cuda" else None


def _moments(a: np.ndarray) -> dict:
    c = _ctx()
    if _gpu_ctx(a.size) is not None:
        from ..ops import analyzers

        m = analyzers.column_moments(a, device=c.device)
        return {"mean": m["mean"], "var": m["std"] ** 2, "min": m["min"], "max": m["max"], "count": int(a.size)}
    return {"mean": float(a.mean()) if a.size else 0.0, "var": float(a.var()) if a.size else 0.0,
            "min": float(a.min()) if a.size else 0.0, "max": float(a.max()) if a.size else 0.0,
            "count": int(a.size)}


# ------------------------------------------------------------------------------ analyzers
def mean(x) -> float:
    a = _num(x)
    return _analyzer("moments", {}, lambda: _moments(a), a)["mean"]


def var(x) -> float:
    a = _num(x)
    return _analyzer("moments", {}, lambda: _moments(a), a)["var"]


def min(x) -> float:  # noqa: A001
    a = _num(x)
    return _analyzer("moments", {}, lambda: _moments(a), a)["min"]


def max(x) -> float:  # noqa: A001
    a = _num(x)
    return _analyzer("moments", {}, lambda: _moments(a), a)["max"]


def size(x) -> int:
    n = len(x) if _is_arrow(x) else int(np.asarray(x).size)
    return _analyzer("size", {}, lambda: n, n)


def sum(x) -> float:  # noqa: A001
    a = _num(x)
    return _analyzer("sum", {}, lambda: float(a.sum()), a)


def quantiles(x, num_buckets: int) -> list[float]:
    a = _num(x)

    def compute():
        """Boundaries = the exact order statistics np.quantile(method="higher") picks at q = 1/nb .. (nb-1)/nb,
        deduplicated. tft's quantiles analyzer is an epsilon-approximate sketch of the same order statistics
        (`taxi_utils.py:128-130`); without TF the exact variant is the pinned definition here. On a GPU: a
        histogram-narrowed selection (csrc/analyzers.hip hist_k / select_k), no sort of the column."""
        if a.size == 0:
            return []
        q = np.arange(1, num_buckets) / num_buckets
        dev = _gpu_ctx(a.size)
        if dev is not None:
            from ..ops import analyzers

            qs = analyzers.quantiles(a, q, method="higher", device=dev)
        else:
            qs = np.quantile(a[~np.isnan(a)], q, method="higher")
        return sorted(set(float(v) for v in qs))

    return _analyzer("quantiles", {"num_buckets": num_buckets}, compute, a)


def vocabulary(x, top_k: int | None = None, frequency_threshold: int | None = None,
               vocab_filename: str | None = None) -> list[str]:
    s = _str_or_arrow(x)

    def compute():
        nonlocal s
        dev = _gpu_ctx(len(s))
        if dev is not None:  # HIP hash-table count (csrc/vocab.hip); identical ordering and cut
            from ..ops import vocab as V

            return V.vocabulary(s, top_k=top_k, frequency_threshold=frequency_threshold, device=dev)
        s = _str(s)
        vals, counts = np.unique(s, return_counts=True)
        order = sorted(zip(counts.tolist(), vals.tolist()), reverse=True)
        if frequency_threshold is not None:
            order = [(c, v) for c, v in order if c >= frequency_threshold]
        if top_k is not None:
            order = order[:top_k]
        return [v for _, v in order]

    return _analyzer("vocabulary", {"top_k": top_k, "frequency_threshold": frequency_threshold,
                                    "vocab_filename": vocab_filename}, compute, s)


# -------------------------------------------------------------------------------- mappers
def scale_to_z_score(x) -> np.ndarray:
    a = _num(x)
    m = _analyzer("moments", {}, lambda: _moments(a), a)
    sd = np.sqrt(m["var"])
    return (a - m["mean"]) / sd if sd > 0 else a - m["mean"]


def scale_to_0_1(x) -> np.ndarray:
    a = _num(x)
    m = _analyzer("moments", {}, lambda: _moments(a), a)
    rng = m["max"] - m["min"]
    return (a - m["min"]) / rng if rng > 0 else np.full_like(a, 0.5)


def scale_by_min_max(x, output_min: float = 0.0, output_max: float = 1.0) -> np.ndarray:
    return scale_to_0_1(x) * (output_max - output_min) + output_min


_FNV_OFF, _FNV_PRIME = 0xCBF29CE484222325, 0x100000001B3


def fingerprint64(s: str) -> int:
    h = _FNV_OFF
    for b in s.encode():
        h = ((h ^ b) * _FNV_PRIME) & 0xFFFFFFFFFFFFFFFF
    return h


def hash_strings(x, hash_buckets: int) -> np.ndarray:
    return np.array([fingerprint64(v) % hash_buckets for v in _str(x)], dtype=np.int64)


def apply_vocabulary(x, vocab: list[str], default_value: int = -1, num_oov_buckets: int = 0) -> np.ndarray:
    s = _str_or_arrow(x)
    dev = _gpu_ctx(len(s))
    if dev is not None:  # device hash-table lookup + FNV OOV buckets (csrc/vocab.hip)
        from ..ops import vocab as V

        return V.apply_vocabulary(s, vocab, default_value=default_value, num_oov_buckets=num_oov_buckets, device=dev)
    s = _str(s)
    index ={v: i for i, v in enumerate(vocab)}
    n = len(vocab)
    out = np.empty(len(s), dtype=np.int64)
    for i, v in enumerate(s):
        j = index.get(v)
        if j is not None:
            out[i] = j
        elif num_oov_buckets > 0:
            out[i] = n + fingerprint64(v) % num_oov_buckets
        else:
            out[i] = default_value
    return out


def compute_and_apply_vocabulary(x, default_value: int = -1, top_k: int | None = None,
                                 frequency_threshold: int | None = None, num_oov_buckets: int = 0,
                                 vocab_filename: str | None = None) -> np.ndarray:
    vocab = vocabulary(x, top_k=top_k, frequency_threshold=frequency_threshold, vocab_filename=vocab_filename)
    return apply_vocabulary(x, vocab, default_value=default_value, num_oov_buckets=num_oov_buckets)


def string_to_int(x, default_value: int = -1, top_k: int | None = None, frequency_threshold: int | None = None,
                  num_oov_buckets: int = 0, vocab_filename: str | None = None) -> np.ndarray:
    """Older tft name used by the KFP taxi module (`kubeflow-pipelines/taxi/preprocessing.py:77-85`)."""
    return compute_and_apply_vocabulary(x, default_value, top_k, frequency_threshold, num_oov_buckets,
                                        vocab_filename)


def apply_buckets(x, boundaries) -> np.ndarray:
    a = _num(x)
    b = np.asarray(boundaries, dtype=np.float64)
    dev = _gpu_ctx(a.size)
    if dev is not None:
        from ..ops import analyzers

        return analyzers.bucketize(a, b, device=dev)
    return np.searchsorted(b, a, side="right").astype(np.int64)


def bucketize(x, num_buckets: int, epsilon: float | None = None) -> np.ndarray:
    return apply_buckets(x, quantiles(x, num_buckets))


def as_string(x) -> np.ndarray:
    if _is_arrow(x) and _arrow_is_str(x):
        return x
    a = np.asarray(_np(x))
    return np.array([str(v) for v in a.tolist()], dtype=object)


def state_summary(state: TransformState) -> list[dict[str, Any]]:
    return [{"kind": e["kind"], **e["params"]} for e in state.entries]
