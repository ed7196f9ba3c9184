"""Sharded (Beam-style) analyze + transform over worker processes.

The reference runs tf.Transform / TFDV / TFMA as Apache Beam pipelines: DirectRunner in-process (`mode='local'`)
or Dataflow (`mode='cloud'`) -- `kubeflow-pipelines/taxi-cab-classification-pipeline.py:52,101,112,133,143`,
`03a_TensorFlow_Transform_Advanced.ipynb` cell 17 (`AnalyzeAndTransformDataset` under `beam.Pipeline`). Every
full-pass analyzer there is a Beam CombineFn: each worker folds its shard into a small accumulator, the
accumulators are merged, and the merged result is broadcast to the mappers.

Here the same structure runs on N local worker processes, each holding one contiguous row shard in memory for the
whole job:

* the user's `preprocessing_fn` is replayed on every shard in a SHARD phase (mifx.transform.api `_analyzer`):
  analyzers already resolved return their merged values, the first unresolved one stops the function and the
  worker returns its accumulator. Analyzers are resolved in call order, so an analyzer whose input depends on
  earlier analyzers (e.g. a vocabulary of a z-scored column) sees exactly the merged values it would in one
  process;
* accumulators -- moments: (count, mean, M2, min, max) merged with Chan et al.'s pairwise update; size / sum:
  totals; vocabulary: per-value counts (then tft's frequency-descending, value-descending order and cut);
  quantiles: an EXACT distributed selection -- per round every shard histograms its values inside each
  quantile's current interval (plus per-bin min / max), the merged histogram narrows the interval to the bin
  holding the rank, and once a bin is small (<= `gather`) its values are gathered and ordered. Boundaries are
  therefore identical to the single-process np.quantile(method="higher") definition (api.quantiles), not a sketch;
* APPLY runs on every shard with the merged state and the outputs are concatenated in shard order -- the same
  rows in the same order as a one-process apply.

    cols, state = analyze_sharded(preprocessing_fn, inputs, num_workers=8)

The Transform component uses it when its `num_workers` (cf. Beam's `--direct_num_workers`) is > 1.
"""
from __future__ import annotations

import multiprocessing as mp
import os
import sys
import traceback

import numpy as np

from . import api

SELECT_BINS = 4096
GATHER = 65536


# ------------------------------------------------------------------------------------------ shards
def _nrows(inputs: dict) -> int:
    lens = {len(v) for v in inputs.values()}
    if len(lens) != 1:
        raise ValueError(f"input columns differ in length: {sorted(lens)}")
    return lens.pop()


def _slice(col, lo: int, hi: int):
    if api._is_arrow(col):
        return col.slice(lo, hi - lo)
    return col[lo:hi]


def shard_inputs(inputs: dict, n: int) -> list[dict]:
    """Contiguous, near-equal row ranges (no empty shard)."""
    rows = _nrows(inputs)
    n = max(1, min(int(n), rows)) if rows else 1
    bounds = np.linspace(0, rows, n + 1).round().astype(np.int64)
    return [{k: _slice(v, int(bounds[i]), int(bounds[i + 1])) for k, v in inputs.items()} for i in range(n)]


# ------------------------------------------------------------------------------------ accumulators
def _moments_acc(a: np.ndarray) -> dict:
    a = np.asarray(a, dtype=np.float64)
    if a.size == 0:
        return {"n": 0, "mean": 0.0, "m2": 0.0, "min": np.inf, "max": -np.inf, "nan": False}
    nan = bool(np.isnan(a).any())
    m = float(a.mean())
    return {"n": int(a.size), "mean": m, "m2": float(((a - m) ** 2).sum()), "min": float(a.min()),
            "max": float(a.max()), "nan": nan}


def _moments_merge(accs: list[dict]) -> dict:
    n, mean, m2 = 0, 0.0, 0.0
    lo, hi, nan = np.inf, -np.inf, False
    for a in accs:
        if a["n"] == 0:
            continue
        nb = a["n"]
        d = a["mean"] - mean
        tot = n + nb
        mean = mean + d * nb / tot
        m2 = m2 + a["m2"] + d * d * n * nb / tot
        n = tot
        lo, hi, nan = min(lo, a["min"]), max(hi, a["max"]), nan or a["nan"]
    if n == 0:
        return {"mean": 0.0, "var": 0.0, "min": 0.0, "max": 0.0, "count": 0}
    if nan:  # numpy semantics of the one-process analyzer: any NaN poisons the moments
        return {"mean": float("nan"), "var": float("nan"), "min": float("nan"), "max": float("nan"), "count": n}
    return {"mean": float(mean), "var": float(m2 / n), "min": float(lo), "max": float(hi), "count": n}


def _value_counts(s) -> dict:
    if api._is_arrow(s):
        import pyarrow as pa
        import pyarrow.compute as pc

        a = s.combine_chunks() if isinstance(s, pa.ChunkedArray) else s
        a = pc.fill_null(a.cast(pa.string()), "")
        vc = pc.value_counts(a)
        return dict(zip(vc.field("values").to_pylist(), vc.field("counts").to_pylist()))
    vals, counts = np.unique(api._str(s), return_counts=True)
    return dict(zip(vals.tolist(), counts.tolist()))


def _vocab_merge(accs: list[dict], params: dict) -> list[str]:
    tot: dict = {}
    for a in accs:
        for k, c in a.items():
            tot[k] = tot.get(k, 0) + int(c)
    order = sorted(((c, v) for v, c in tot.items()), reverse=True)
    if params.get("frequency_threshold") is not None:
        order = [(c, v) for c, v in order if c >= params["frequency_threshold"]]
    if params.get("top_k") is not None:
        order = order[: params["top_k"]]
    return [v for _, v in order]


# worker-side quantile rounds: the analyzer's input (non-NaN) is cached per analyzer index
def _q_init(a: np.ndarray) -> dict:
    """Count, FINITE min / max and the +-inf counts of the non-NaN input: the selection rounds bin the finite range
    only (linspace over an infinite interval is NaN everywhere); ranks in the infinite tails resolve directly."""
    a = a[~np.isnan(a)]
    fin = a[np.isfinite(a)]
    return {"n": int(a.size), "min": float(fin.min()) if fin.size else np.inf,
            "max": float(fin.max()) if fin.size else -np.inf,
            "ninf": int(np.count_nonzero(a == -np.inf)), "pinf": int(np.count_nonzero(a == np.inf))}


def _q_hist(a: np.ndarray, intervals: list) -> list:
    """Per interval [lo, hi] (closed): SELECT_BINS-bin counts over linspace(lo, hi) and per-bin min / max."""
    out = []
    for lo, hi in intervals:
        v = a[(a >= lo) & (a <= hi)]
        edges = np.linspace(lo, hi, SELECT_BINS + 1)
        b = np.clip(np.searchsorted(edges[1:-1], v, side="right"), 0, SELECT_BINS - 1)
        cnt = np.bincount(b, minlength=SELECT_BINS)
        bmin = np.full(SELECT_BINS, np.inf)
        bmax = np.full(SELECT_BINS, -np.inf)
        np.minimum.at(bmin, b, v)
        np.maximum.at(bmax, b, v)
        out.append((cnt, bmin, bmax))
    return out


def _q_gather(a: np.ndarray, intervals: list) -> list:
    return [np.sort(a[(a >= lo) & (a <= hi)]) for lo, hi in intervals]


# ------------------------------------------------------------------------------------------ workers
def _run_to(fn, inputs: dict, resolved: list):
    """Replay fn in the SHARD phase: returns the ShardStop of the first unresolved analyzer, or None."""
    st = api.TransformState(list(resolved))
    try:
        with api._phase("shard", st):
            fn(dict(inputs))
    except api.ShardStop as stop:
        return stop
    return None


def _worker(conn, fn_bytes: bytes, inputs: dict) -> None:
    import cloudpickle

    fn = cloudpickle.loads(fn_bytes)
    cache: dict = {}  # analyzer index -> its (non-NaN float64) input, for the quantile rounds
    while True:
        msg = conn.recv()
        try:
            op = msg[0]
            if op == "stop":
                conn.send(("ok", None))
                return
            if op == "acc":
                _, idx, resolved = msg
                stop = _run_to(fn, inputs, resolved)
                if stop is None:
                    conn.send(("ok", None))
                    continue
                if stop.kind == "moments":
                    acc = _moments_acc(stop.data)
                elif stop.kind == "size":
                    acc = int(stop.data)
                elif stop.kind == "sum":
                    acc = float(np.asarray(stop.data, dtype=np.float64).sum())
                elif stop.kind == "vocabulary":
                    acc = _value_counts(stop.data)
                elif stop.kind == "quantiles":
                    a = np.asarray(stop.data, dtype=np.float64)
                    cache[idx] = a[~np.isnan(a)]
                    acc = _q_init(a)
                else:
                    raise NotImplementedError(f"no sharded accumulator for analyzer {stop.kind!r}")
                conn.send(("ok", (stop.kind, stop.params, acc)))
            elif op == "qhist":
                conn.send(("ok", _q_hist(cache[msg[1]], msg[2])))
            elif op == "qgather":
                conn.send(("ok", _q_gather(cache[msg[1]], msg[2])))
            elif op == "apply":
                cache.clear()
                conn.send(("ok", api.apply(fn, inputs, api.TransformState(list(msg[1])))))
            else:
                raise ValueError(f"unknown op {op!r}")
        except Exception:  # noqa: BLE001 -- reported to the driver
            conn.send(("err", traceback.format_exc()))


class ShardWorkers:
    """N worker processes, one shard each (spawned: no inherited GPU or thread state)."""

    def __init__(self, fn, shards: list[dict]):
        import cloudpickle

        ctx = mp.get_context("spawn")
        mod = sys.modules.get(getattr(fn, "__module__", "") or "")
        if mod is not None and mod.__name__.startswith("mifx_user_"):
            # a module file loaded by path (import_module_file): not importable by name in the workers
            cloudpickle.register_pickle_by_value(mod)
        fb = cloudpickle.dumps(fn)
        self.conns, self.procs = [], []
        for sh in shards:
            a, b = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(b, fb, sh), daemon=True)
            p.start()
            b.close()
            self.conns.append(a)
            self.procs.append(p)

    def call(self, msg, per_worker: list | None = None) -> list:
        for i, c in enumerate(self.conns):
            c.send(per_worker[i] if per_worker is not None else msg)
        out = []
        for c in self.conns:
            status, val = c.recv()
            if status != "ok":
                raise RuntimeError(f"transform worker failed:\n{val}")
            out.append(val)
        return out

    def close(self) -> None:
        for c in self.conns:
            try:
                c.send(("stop",))
                c.recv()
            except (EOFError, OSError, BrokenPipeError):
                pass
        for p in self.procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        self.conns, self.procs = [], []


# ------------------------------------------------------------------------------------------ driver
def _ranks_higher(n: int, num_buckets: int) -> np.ndarray:
    from ..ops.analyzers import _virtual_index

    q = np.arange(1, num_buckets) / num_buckets
    return np.clip(np.ceil(_virtual_index(n, q)), 0, n - 1).astype(np.int64)


def _distributed_order_stats(workers: ShardWorkers, idx: int, inits: list[dict], ranks: np.ndarray) -> np.ndarray:
    lo = min(a["min"] for a in inits)
    hi = max(a["max"] for a in inits)
    n = sum(a["n"] for a in inits)
    ninf = sum(a.get("ninf", 0) for a in inits)
    pinf = sum(a.get("pinf", 0) for a in inits)
    out = np.full(ranks.size, np.nan)
    # ranks in the infinite tails need no selection; the rest select among the finite values in [lo, hi]
    state = {}
    for j in range(ranks.size):
        if ranks[j] < ninf:
            out[j] = -np.inf
        elif ranks[j] >= n - pinf:
            out[j] = np.inf
        else:  # per pending rank: [lo, hi] (closed) holds it; `below` values (the -inf ones first) lie under lo
            state[j] = [lo, hi, ninf]
    while state:
        pend = sorted(state)
        done = [j for j in pend if state[j][0] == state[j][1]]
        for j in done:
            out[j] = state.pop(j)[0]
        pend = [j for j in pend if j in state]
        if not pend:
            break
        hists = workers.call(("qhist", idx, [tuple(state[j][:2]) for j in pend]))
        gather = []
        for k, j in enumerate(pend):
            cnt = sum(h[k][0] for h in hists)
            bmin = np.min([h[k][1] for h in hists], axis=0)
            bmax = np.max([h[k][2] for h in hists], axis=0)
            below = state[j][2]
            cum = below + np.cumsum(cnt)
            b = int(np.searchsorted(cum, ranks[j], side="right"))
            nb_below = int(cum[b - 1]) if b > 0 else below
            state[j] = [float(bmin[b]), float(bmax[b]), nb_below]
            if bmin[b] == bmax[b]:
                continue  # resolved next round
            if cnt[b] <= GATHER:
                gather.append(j)
        if gather:
            vals = workers.call(("qgather", idx, [tuple(state[j][:2]) for j in gather]))
            for k, j in enumerate(gather):
                v = np.sort(np.concatenate([w[k] for w in vals]))
                out[j] = v[ranks[j] - state[j][2]]
                del state[j]
    return out


def _resolve(workers: ShardWorkers, idx: int, kind: str, params: dict, accs: list):
    if kind == "moments":
        return _moments_merge(accs)
    if kind == "size":
        return int(sum(accs))
    if kind == "sum":
        return float(sum(accs))
    if kind == "vocabulary":
        return _vocab_merge(accs, params)
    if kind == "quantiles":
        n = sum(a["n"] for a in accs)
        if n == 0:
            return []
        qs = _distributed_order_stats(workers, idx, accs, _ranks_higher(n, params["num_buckets"]))
        return sorted(set(float(v) for v in qs))
    raise NotImplementedError(kind)


def analyze_sharded(preprocessing_fn, inputs: dict, num_workers: int | None = None,
                    transform: bool = True) -> tuple[dict | None, api.TransformState]:
    """Beam-style analyze (+ transform of the same data) over `num_workers` processes; same contract as
    mifx.transform.analyze. num_workers defaults to the CPU count (cf. `--direct_num_workers=0`)."""
    n = int(num_workers or os.cpu_count() or 1)
    shards = shard_inputs(inputs, n)
    workers = ShardWorkers(preprocessing_fn, shards)
    try:
        resolved: list = []
        while True:
            replies = workers.call(("acc", len(resolved), resolved))
            live = [r for r in replies if r is not None]
            if not live:
                break
            if len(live) != len(replies) or len({(r[0], repr(r[1])) for r in live}) != 1:
                raise RuntimeError("shards disagree on the analyzer sequence (data-dependent control flow in "
                                   "preprocessing_fn)")
            kind, params = live[0][0], live[0][1]
            values = _resolve(workers, len(resolved), kind, params, [r[2] for r in live])
            resolved.append({"kind": kind, "params": params, "values": values})
        state = api.TransformState(resolved)
        cols = None
        if transform:
            parts = workers.call(("apply", resolved))
            cols = {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
        return cols, state
    finally:
        workers.close()


def transform_sharded(preprocessing_fn, inputs: dict, state: api.TransformState,
                      num_workers: int | None = None) -> dict:
    """APPLY over `num_workers` processes (row order preserved)."""
    shards = shard_inputs(inputs, int(num_workers or os.cpu_count() or 1))
    workers = ShardWorkers(preprocessing_fn, shards)
    try:
        parts = workers.call(("apply", state.entries))
        return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]}
    finally:
        workers.close()
