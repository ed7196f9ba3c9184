"""HIP analyzer kernels (column moments, bucketize, sliced-metric histograms) vs numpy fp64."""
import numpy as np
import pytest

from mifx.ops import analyzers as an


@pytest.mark.gpu
def test_column_moments_matches_numpy():
    r = np.random.default_rng(0)
    x = r.normal(3.0, 2.0, 1_000_003)
    x[::97] = np.nan
    x[::101] = 0.0
    got = an.column_moments(x, device="cuda")
    ref = an.column_moments(x, device=None)
    assert got["count"] == ref["count"] and got["zeros"] == ref["zeros"]
    for k in ("mean", "std", "min", "max"):
        assert got[k] == pytest.approx(ref[k], rel=1e-10, abs=1e-12), k


@pytest.mark.gpu
def test_bucketize_matches_searchsorted():
    r = np.random.default_rng(1)
    x = r.normal(size=300_001)
    b = np.quantile(x, np.arange(1, 10) / 10)
    x[:10] = b[:10 - 1].tolist() + [b[-1]]  # exact boundary hits go to the upper bucket
    assert np.array_equal(an.bucketize(x, b, device="cuda"), np.searchsorted(b, x, side="right"))


@pytest.mark.gpu
def test_segment_hist_matches_numpy():
    r = np.random.default_rng(2)
    n, ns = 200_000, 24
    seg = r.integers(0, ns, n)
    y = (r.random(n) < 0.3).astype(np.float32)
    p = np.clip(r.random(n) * 0.6 + y * 0.3, 0, 1).astype(np.float32)
    s_g, h_g = an.segment_hist(seg, y, p, ns, 1000, device="cuda")
    s_c, h_c = an.segment_hist(seg, y, p, ns, 1000, device=None)
    assert np.array_equal(h_g, h_c)
    assert np.allclose(s_g, s_c, rtol=1e-9)
    auc = an.auc_from_hist(h_c[0])
    assert 0.5 < auc < 1.0
