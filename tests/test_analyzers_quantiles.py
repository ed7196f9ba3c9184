"""Exact quantiles / histograms / value counts for Transform (KN8) and StatisticsGen (KN11): the GPU path
(csrc/analyzers.hip hist_k + select_k: histogram-narrowed order statistics, no device sort) and the host path
must both be bit-identical to numpy (np.quantile "higher" / "linear", np.histogram, np.unique). The Transform's
bucketize boundaries are exact "higher" order statistics; tft's own quantiles analyzer is an epsilon-approximate
sketch of these (`airflow-dags/taxi_utils.py:128-130`) -- that parity is unpinned without TF."""
import numpy as np
import pyarrow as pa
import pytest
import torch

from mifx.ops import analyzers as A


def _cases(rng):
    yield rng.normal(size=1001)
    yield rng.integers(0, 5, 4000).astype(np.float64)  # duplicates
    yield np.full(77, 3.25)  # constant
    yield np.array([2.0])
    yield np.concatenate([rng.normal(size=300), [np.nan] * 7])
    yield np.concatenate([rng.normal(size=2000), rng.normal(1e6, 1, 5)])  # outliers: crowded low bins


def test_host_quantiles_match_numpy_bitwise():
    rng = np.random.default_rng(0)
    for a in _cases(rng):
        v = a[~np.isnan(a)]
        for q in (np.linspace(0, 1, 11), np.arange(1, 10) / 10, rng.random(31)):
            for m in ("higher", "linear"):
                assert np.array_equal(A.quantiles(a, q, m), np.quantile(v, q, method=m)), (m, a.size)


def test_host_histogram_and_value_counts():
    rng = np.random.default_rng(1)
    a = rng.gamma(2, 3, 5000)
    e = np.linspace(a.min(), a.max(), 11)
    assert np.array_equal(A.histogram(a, e), np.histogram(a, bins=e)[0])
    ints = rng.integers(-3, 40, 3000)
    u, c = A.int_value_counts(ints)
    uu, cc = np.unique(ints, return_counts=True)
    assert np.array_equal(u, uu) and np.array_equal(c, cc)


@pytest.mark.gpu
def test_gpu_quantiles_match_numpy_bitwise():
    rng = np.random.default_rng(2)
    for a in list(_cases(rng)) + [rng.normal(41.9, 0.05, 1 << 20)]:
        v = a[~np.isnan(a)]
        for q in (np.linspace(0, 1, 11), np.arange(1, 10) / 10, rng.random(17)):
            for m in ("higher", "linear"):
                got = A.quantiles(a, q, m, device="cuda")
                assert np.array_equal(got, np.quantile(v, q, method=m)), (m, a.size)
    ks = np.array([0, 5, 999, 500])
    a = rng.normal(size=1000)
    assert np.array_equal(A.order_statistics(a, ks, device="cuda"), np.sort(a)[ks])


@pytest.mark.gpu
def test_gpu_histogram_edges_and_int_counts():
    rng = np.random.default_rng(3)
    a = np.round(rng.gamma(2, 3, 100000), 1)  # many values exactly on the edges
    for e in (np.linspace(a.min(), a.max(), 11), np.arange(0.0, 30.0, 0.5), np.array([1.0, 2.0])):
        assert np.array_equal(A.histogram(a, e, device="cuda"), np.histogram(a, bins=e)[0])
    ints = rng.integers(-1000, 100000, 200000)
    u, c = A.int_value_counts(ints, device="cuda")
    uu, cc = np.unique(ints, return_counts=True)
    assert np.array_equal(u, uu) and np.array_equal(c, cc)


@pytest.mark.gpu
def test_gpu_statistics_equal_host_statistics():
    from mifx.data_validation import stats as S

    rng = np.random.default_rng(4)
    n = 50000
    names = np.array(["Cash", "Credit Card", "Dispute", "No Charge", "Ünknown"], dtype=object)
    t = pa.table({"fare": pa.array(np.where(rng.random(n) < 0.01, np.nan, rng.gamma(2, 6, n))),
                  "hour": pa.array(rng.integers(0, 24, n)),
                  "payment_type": pa.array([None if i % 97 == 0 else s for i, s in
                                            enumerate(names[rng.integers(0, 5, n)])])})
    g, h = S.generate_statistics_from_table(t, "x", device="cuda"), S.generate_statistics_from_table(t, "x")
    # histograms, quantiles, median, counts and string statistics are bit-identical; mean / std_dev come from the
    # fp64 Welford reduction (another summation order than numpy's pairwise sum): equal to ~1e-15 relative
    _same(g, h)


def _same(a, b, path=""):
    if isinstance(a, dict):
        assert set(a) == set(b), path
        for k in a:
            _same(a[k], b[k], f"{path}.{k}")
    elif isinstance(a, list):
        assert len(a) == len(b), path
        for i, (x, y) in enumerate(zip(a, b)):
            _same(x, y, f"{path}[{i}]")
    elif isinstance(a, float) and path.rsplit(".", 1)[-1] in ("mean", "std_dev"):
        assert a == pytest.approx(b, rel=1e-12, abs=1e-12), path
    else:
        assert a == b, (path, a, b)


@pytest.mark.gpu
def test_transform_bucketize_boundaries_on_gpu_equal_host(monkeypatch):
    import mifx.transform as mt
    import mifx.transform.api as tapi

    rng = np.random.default_rng(5)
    lat = rng.normal(41.9, 0.05, 20000)

    def fn(inputs):
        return {"b": mt.bucketize(inputs["lat"], 10)}

    monkeypatch.setattr(tapi, "GPU_MIN_ROWS", 0)
    out_g, st_g = mt.analyze(fn, {"lat": lat}, device="cuda")
    out_c, st_c = mt.analyze(fn, {"lat": lat}, device=None)
    assert np.array_equal(out_g["b"], out_c["b"])
    assert st_g.to_dict() == st_c.to_dict() if hasattr(st_g, "to_dict") else True


def _inf_case(rng):
    a = np.concatenate([rng.normal(size=700), [np.inf] * 3, [-np.inf] * 5, [np.nan] * 2])
    rng.shuffle(a)
    return a


def test_host_order_statistics_with_infinities():
    rng = np.random.default_rng(11)
    a = _inf_case(rng)
    v = np.sort(a[~np.isnan(a)])
    ks = np.array([0, 4, 5, 6, 300, 704, 705, 707])
    assert np.array_equal(A.order_statistics(a, ks), v[ks])
    q = np.linspace(0, 1, 11)
    assert np.array_equal(A.quantiles(a, q, "higher"), np.quantile(v, q, method="higher"))


@pytest.mark.gpu
def test_gpu_order_statistics_with_infinities():
    """+-inf values: the tails resolve directly, the histogram selection runs over the finite values (an infinite
    range would make every bin edge NaN)."""
    rng = np.random.default_rng(11)
    a = _inf_case(rng)
    v = np.sort(a[~np.isnan(a)])
    ks = np.array([0, 4, 5, 6, 300, 704, 705, 707])
    assert np.array_equal(A.order_statistics(a, ks, device="cuda"), v[ks])
    q = np.linspace(0, 1, 11)
    assert np.array_equal(A.quantiles(a, q, "higher", device="cuda"), np.quantile(v, q, method="higher"))
    allinf = np.array([np.inf, -np.inf, np.inf])
    assert np.array_equal(A.order_statistics(allinf, np.array([0, 1, 2]), device="cuda"), np.sort(allinf))
