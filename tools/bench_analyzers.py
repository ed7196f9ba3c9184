"""Transform-analyzer microbench on a taxi-shaped synthetic table: GPU HIP kernels (vocabulary
count + lookup, z-score moments, quantile bucketize) vs the host numpy/Python path, same outputs.

    python tools/bench_analyzers.py [--rows N]     -> one JSON line per analyzer
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.ops import analyzers, vocab  # noqa: E402


def _t(fn, reps=3):
    fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1 << 20)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    n = a.rows
    companies = np.array([f"company_{i:04d}" for i in range(5000)] + ["Cash", "Credit Card", ""], dtype=object)
    p = 1.0 / np.arange(1, len(companies) + 1) ** 1.2
    col = companies[rng.choice(len(companies), size=n, p=p / p.sum())].tolist()
    fare = rng.gamma(2.0, 6.0, n)
    lat = rng.normal(41.9, 0.05, n)
    dev = "cuda" if torch.cuda.is_available() else None
    res = []

    tg, vg = _t(lambda: vocab.vocabulary(col, top_k=1000, device=dev))
    tc, vc = _t(lambda: vocab.vocabulary(col, top_k=1000, device=None), reps=1)
    assert vg == vc
    res.append({"op": "vocabulary(top_k=1000)", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    import pyarrow as pa

    arr = pa.array(col)  # the Transform component's GPU input form (Arrow string column)
    tg, va = _t(lambda: vocab.vocabulary(arr, top_k=1000, device=dev))
    assert va == vc
    res.append({"op": "vocabulary(top_k=1000) [arrow input]", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    dv = vocab.DeviceVocabulary(vg, dev) if dev else None
    if dv is not None:
        tg, ia = _t(lambda: dv.lookup(arr, -1, 10))
        res.append({"op": "apply_vocabulary(oov=10) [arrow input]", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": None})
    tg, ig = _t(lambda: dv.lookup(col, -1, 10) if dv else vocab.apply_vocabulary(col, vg, -1, 10))
    tc, ic = _t(lambda: vocab.apply_vocabulary(col, vg, -1, 10, device=None), reps=1)
    assert np.array_equal(ig, ic)
    if dv is not None:
        assert np.array_equal(ia, ic)
    res.append({"op": "apply_vocabulary(oov=10)", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    tg, mg = _t(lambda: analyzers.column_moments(fare, device=dev))
    tc, mc = _t(lambda: analyzers.column_moments(fare, device=None))
    assert abs(mg["mean"] - mc["mean"]) < 1e-9 * abs(mc["mean"]) + 1e-12
    res.append({"op": "scale_to_z_score moments", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    bnd = np.quantile(lat, np.arange(1, 10) / 10, method="higher")
    tg, bg = _t(lambda: analyzers.bucketize(lat, bnd, device=dev))
    tc, bc = _t(lambda: analyzers.bucketize(lat, bnd, device=None))
    assert np.array_equal(bg, bc)
    res.append({"op": "bucketize(10)", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    qs = np.arange(1, 10) / 10
    if dev:
        tl = torch.from_numpy(lat).to(dev)  # column already on the device (Transform / TFDV GPU path)
        tg, qg = _t(lambda: analyzers.quantiles(tl, qs, method="higher", device=dev))
    else:
        tg, qg = _t(lambda: analyzers.quantiles(lat, qs, method="higher"))
    tc, qc = _t(lambda: np.quantile(lat, qs, method="higher"))
    assert np.array_equal(qg, qc)
    res.append({"op": "quantiles(10, method=higher) exact", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})
    dup = rng.integers(0, 7, n).astype(np.float64)  # heavy duplicates: crowded bins
    tg, qg = _t(lambda: analyzers.quantiles(dup, np.linspace(0, 1, 11), device=dev))
    tc, qc = _t(lambda: np.quantile(dup, np.linspace(0, 1, 11)))
    assert np.array_equal(qg, qc)
    res.append({"op": "quantiles(linspace 11) duplicates", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})
    edges = np.linspace(fare.min(), fare.max(), 11)
    tg, hg = _t(lambda: analyzers.histogram(fare, edges, device=dev))
    tc, hc = _t(lambda: np.histogram(fare, bins=edges)[0])
    assert np.array_equal(hg, hc)
    res.append({"op": "histogram(10 equal-width)", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})

    from mifx.data_validation import stats as S

    tbl = pa.table({"fare": fare, "pickup_latitude": lat, "trip_start_hour": rng.integers(0, 24, n),
                    "company": arr})
    tg, sg = _t(lambda: S.generate_statistics_from_table(tbl, device=dev), reps=2)
    tc, sc = _t(lambda: S.generate_statistics_from_table(tbl, device=None), reps=1)
    fg = {f["name"]: f for f in sg["datasets"][0]["features"]}
    for f in sc["datasets"][0]["features"]:  # exact except the Welford mean / std (ulps)
        a, b = fg[f["name"]], f
        for k in ("histograms", "median", "min", "max", "num_zeros", "value_counts", "top_values", "unique"):
            sa, sb = a.get("num_stats", a.get("string_stats")), b.get("num_stats", b.get("string_stats"))
            assert sa.get(k) == sb.get(k), (f["name"], k)
    res.append({"op": "TFDV generate_statistics (4 columns)", "rows": n, "gpu_ms": 1e3 * tg, "cpu_ms": 1e3 * tc})
    for r in res:
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
