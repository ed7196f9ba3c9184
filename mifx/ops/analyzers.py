"""Analyzer / evaluation kernels (csrc/analyzers.hip) with numpy reference implementations.

`device` is a torch device (or string). On a CUDA/HIP device the native kernels are REQUIRED
(no silent fallback); on CPU the numpy path runs."""
from __future__ import annotations

import ctypes
import functools

import numpy as np
import torch

from . import _lib
from ._lib import I32, I64, VP, check, ptr, sig, stream_handle


def _is_gpu(device) -> bool:
    return device is not None and torch.device(device).type == "cuda"


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("analyzers")
    return {
        "moments": sig(lib, "mifx_an_moments", [VP, I64, VP, I32, VP, VP]),
        "mbytes": sig(lib, "mifx_an_moments_partial_bytes", []),
        "bucketize": sig(lib, "mifx_an_bucketize", [VP, I64, VP, I32, VP, VP]),
        "seghist": sig(lib, "mifx_an_segment_hist", [VP, VP, VP, I64, I32, I32, VP, VP, VP]),
        "hist": sig(lib, "mifx_an_histogram", [VP, I64, I32, VP, ctypes.c_double, ctypes.c_double, I32, VP, VP]),
        "select": sig(lib, "mifx_an_select", [VP, I64, ctypes.c_double, ctypes.c_double, I32, VP, I32, VP, VP, VP]),
    }


def column_moments(x, device=None) -> dict:
    if torch.is_tensor(x) and _is_gpu(device):  # already on the device: no host round trip
        a = x
    else:
        a = np.asarray(x.cpu() if torch.is_tensor(x) else x, dtype=np.float64)
    if not _is_gpu(device):
        v = a[~np.isnan(a)]
        if v.size == 0:
            return {"count": 0, "mean": 0.0, "std": 0.0, "min": 0.0, "max": 0.0, "zeros": 0}
        return {"count": int(v.size), "mean": float(v.mean()), "std": float(v.std()), "min": float(v.min()),
                "max": float(v.max()), "zeros": int((v == 0).sum())}
    dev = torch.device(device)
    t = _dev_f64(a, dev)
    grid = int(max(1, min(1024, (t.numel() + 255) // 256)))
    part = torch.empty(grid * _fns()["mbytes"](), dtype=torch.uint8, device=dev)
    out = torch.empty(6, dtype=torch.float64, device=dev)
    check(_fns()["moments"](ptr(t), t.numel(), ptr(part), grid, ptr(out), stream_handle(dev)), "mifx_an_moments")
    n, mean, var, mn, mx, zeros = out.cpu().tolist()
    if n == 0:
        return {"count": 0, "mean": 0.0, "std": 0.0, "min": 0.0, "max": 0.0, "zeros": 0}
    return {"count": int(n), "mean": mean, "std": float(np.sqrt(max(var, 0.0))), "min": mn, "max": mx,
            "zeros": int(zeros)}


def bucketize(x, boundaries, device=None) -> np.ndarray:
    a = np.asarray(x, dtype=np.float64)
    b = np.asarray(boundaries, dtype=np.float64)
    if not _is_gpu(device) or b.size > 1024:
        return np.searchsorted(b, a, side="right").astype(np.int64)
    dev = torch.device(device)
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    tb = torch.from_numpy(np.ascontiguousarray(b)).to(dev)
    out = torch.empty(a.size, dtype=torch.int64, device=dev)
    check(_fns()["bucketize"](ptr(t), a.size, ptr(tb), b.size, ptr(out), stream_handle(dev)), "mifx_an_bucketize")
    return out.cpu().numpy()


def segment_hist(seg, label, prob, num_segments: int, num_buckets: int = 1000, device=None):
    """Per-segment [count, label_sum, pred_sum, loss_sum, correct] and label-split prob histograms."""
    seg = np.asarray(seg, np.int32)
    y = np.asarray(label, np.float32)
    p = np.asarray(prob, np.float32)
    if not _is_gpu(device):
        sums = np.zeros((num_segments, 5))
        hist = np.zeros((num_segments, num_buckets, 2), np.int64)
        pc = np.clip(p, 1e-7, 1 - 1e-7).astype(np.float64)
        b = np.minimum((pc * num_buckets).astype(np.int64), num_buckets - 1)
        loss = -(y * np.log(pc) + (1 - y) * np.log(1 - pc))
        ok = (seg >= 0) & (seg < num_segments)
        s, yb = seg[ok], (y[ok] > 0.5).astype(np.int64)
        np.add.at(hist, (s, b[ok], yb), 1)
        for j, v in enumerate([np.ones(ok.sum()), y[ok], pc[ok], loss[ok], ((pc[ok] > 0.5) == (y[ok] > 0.5))]):
            np.add.at(sums[:, j], s, v)
        return sums, hist
    dev = torch.device(device)
    ts, ty, tp = (torch.from_numpy(np.ascontiguousarray(v)).to(dev) for v in (seg, y, p))
    sums = torch.zeros(num_segments, 5, dtype=torch.float64, device=dev)
    hist = torch.zeros(num_segments, num_buckets, 2, dtype=torch.int32, device=dev)
    check(_fns()["seghist"](ptr(ts), ptr(ty), ptr(tp), seg.size, num_segments, num_buckets, ptr(sums), ptr(hist),
                            stream_handle(dev)), "mifx_an_segment_hist")
    return sums.cpu().numpy(), hist.cpu().numpy().astype(np.int64)


def auc_from_hist(h: np.ndarray) -> float:
    """Trapezoidal ROC AUC from a [num_buckets, 2] (neg, pos) prediction histogram."""
    neg, pos = h[:, 0][::-1].astype(np.float64), h[:, 1][::-1].astype(np.float64)
    tp, fp = np.cumsum(pos), np.cumsum(neg)
    if tp[-1] == 0 or fp[-1] == 0:
        return float("nan")
    tpr = np.concatenate([[0], tp / tp[-1]])
    fpr = np.concatenate([[0], fp / fp[-1]])
    return float(np.trapezoid(tpr, fpr) if hasattr(np, "trapezoid") else np.trapz(tpr, fpr))


def _dev_f64(x, device):
    if torch.is_tensor(x):
        return x.to(device=device, dtype=torch.float64).contiguous()
    return torch.from_numpy(np.ascontiguousarray(np.asarray(x, dtype=np.float64))).to(device)


def histogram(x, edges, device=None) -> np.ndarray:
    """np.histogram(x, bins=edges)[0] (NaNs dropped; the last bin closed), int64 counts. GPU: one LDS-privatised
    pass with the edges searched per element (csrc/analyzers.hip hist_k, mode 0)."""
    e = np.asarray(edges, dtype=np.float64)
    nb = e.size - 1
    if not _is_gpu(device) or nb > 4096 or nb < 1:
        a = np.asarray(x.cpu() if torch.is_tensor(x) else x, dtype=np.float64)
        return np.histogram(a[~np.isnan(a)], bins=e)[0].astype(np.int64)
    dev = torch.device(device)
    t = _dev_f64(x, dev)
    te = torch.from_numpy(e).to(dev)
    out = torch.zeros(nb, dtype=torch.int64, device=dev)
    check(_fns()["hist"](ptr(t), t.numel(), 0, ptr(te), 0.0, 0.0, nb, ptr(out), stream_handle(dev)),
          "mifx_an_histogram")
    return out.cpu().numpy()


def _uniform_hist(t, lo: float, inv: float, nb: int) -> torch.Tensor:
    out = torch.zeros(nb, dtype=torch.int64, device=t.device)
    check(_fns()["hist"](ptr(t), t.numel(), 1, None, float(lo), float(inv), int(nb), ptr(out),
                         stream_handle(t.device)), "mifx_an_histogram(uniform)")
    return out


def int_value_counts(x, device=None, max_range: int = 1 << 20):
    """(values, counts) of an integer column: a unit-bin histogram over [min, max] on the GPU when the range is at
    most max_range (exact: integer-valued doubles), else np.unique."""
    a = np.asarray(x, dtype=np.int64)
    if a.size == 0:
        return a, a
    lo, hi = int(a.min()), int(a.max())
    if not _is_gpu(device) or hi - lo + 1 > max_range or abs(lo) > 2**52 or abs(hi) > 2**52:
        return np.unique(a, return_counts=True)
    dev = torch.device(device)
    t = _dev_f64(a, dev)
    c = _uniform_hist(t, float(lo), 1.0, hi - lo + 1).cpu().numpy()
    nz = np.nonzero(c)[0]
    return nz + lo, c[nz]


SELECT_BINS = 16384
SELECT_CAP = 65536


def order_statistics(x, ks, device=None) -> np.ndarray:
    """The k-th smallest values (0-based ranks ks) of the non-NaN entries of x, exactly. GPU: a 16384-bin uniform
    histogram over [min, max] places every rank in one bin, the values of those bins are gathered (select_k) and
    ordered on the host -- a few hundred values for 1M rows instead of a device sort of the whole column."""
    ks = np.asarray(ks, dtype=np.int64)
    if not _is_gpu(device):
        a = np.asarray(x.cpu() if torch.is_tensor(x) else x, dtype=np.float64)
        a = a[~np.isnan(a)]
        return np.partition(a, ks)[ks] if ks.size else np.zeros(0)
    dev = torch.device(device)
    t = _dev_f64(x, dev)
    t = t[~torch.isnan(t)]
    n = t.numel()
    if ks.size == 0:
        return np.zeros(0)
    if ks.min() < 0 or ks.max() >= n:
        raise IndexError("rank out of range")
    # +-inf: ranks in the infinite tails resolve directly; the histogram selection runs over the finite values
    ninf, pinf = int((t == -np.inf).sum()), int((t == np.inf).sum())
    if ninf or pinf:
        res = np.empty(ks.size)
        lo_tail, hi_tail = ks < ninf, ks >= n - pinf
        res[lo_tail], res[hi_tail] = -np.inf, np.inf
        mid = ~(lo_tail | hi_tail)
        if mid.any():
            res[mid] = order_statistics(t[torch.isfinite(t)], ks[mid] - ninf, device)
        return res
    lo, hi = (float(v) for v in torch.aminmax(t))
    if hi == lo:
        return np.full(ks.size, lo)
    nb = SELECT_BINS
    inv = nb / (hi - lo)
    # the max itself maps to bin nb when (hi - lo) * inv rounds up to nb: widen the top edge by one ulp's worth
    while (hi - lo) * inv >= nb:
        inv = np.nextafter(inv, 0.0)
    cum = np.cumsum(_uniform_hist(t, lo, inv, nb).cpu().numpy())
    bins = np.searchsorted(cum, ks, side="right")
    first = np.concatenate([[0], cum])[bins]
    targets = np.unique(bins)
    slot = np.full(nb, -1, dtype=np.int32)
    slot[targets] = np.arange(targets.size, dtype=np.int32)
    sizes = (cum[targets] - np.concatenate([[0], cum])[targets]).astype(np.int64)
    cap = int(max(1, min(SELECT_CAP, sizes.max())))
    if sizes.max() > SELECT_CAP:  # a crowded bin (duplicates / clusters): gather exactly its count
        cap = int(sizes.max())
    ts = torch.from_numpy(slot).to(dev)
    cnt = torch.zeros(targets.size, dtype=torch.int32, device=dev)
    out = torch.empty(targets.size * cap, dtype=torch.float64, device=dev)
    check(_fns()["select"](ptr(t), n, float(lo), float(inv), nb, ptr(ts), cap, ptr(cnt), ptr(out),
                           stream_handle(dev)), "mifx_an_select")
    got = cnt.cpu().numpy()
    assert np.array_equal(got, sizes), (got, sizes)
    vals = out.view(targets.size, cap).cpu().numpy()
    res = np.empty(ks.size)
    for i, (k, b) in enumerate(zip(ks, bins)):
        j = int(slot[b])
        res[i] = np.sort(vals[j, :sizes[j]])[k - first[i]]
    return res


def _virtual_index(n: int, q: np.ndarray) -> np.ndarray:
    # numpy's virtual index for "linear" / "higher" (numpy 2.x _QuantileMethods: (n - 1) * q)
    return (n - 1) * q


def quantiles(x, qs, method: str = "linear", device=None) -> np.ndarray:
    """np.quantile(x[~nan], qs, method=...) for "higher" and "linear": numpy's virtual index and lerp on exact order
    statistics, so bit-identical to numpy on both the CPU and the GPU path (tests/test_analyzers_quantiles.py)."""
    q = np.asarray(qs, dtype=np.float64)
    if _is_gpu(device):
        t = _dev_f64(x, torch.device(device))
        n = int((~torch.isnan(t)).sum())
    else:
        t = np.asarray(x.cpu() if torch.is_tensor(x) else x, dtype=np.float64)
        t = t[~np.isnan(t)]
        n = t.size
    if n == 0:
        return np.full(q.shape, np.nan)
    vi = _virtual_index(n, q)
    if method == "higher":
        idx = np.clip(np.ceil(vi), 0, n - 1).astype(np.int64)
        return order_statistics(t, idx, device)
    if method != "linear":
        raise ValueError(f"unsupported quantile method {method}")
    prev = np.clip(np.floor(vi), 0, n - 1).astype(np.int64)
    nxt = np.clip(prev + 1, 0, n - 1)
    gamma = vi - np.floor(vi)
    gamma = np.where(vi < 0, 0.0, np.where(vi > n - 1, 0.0, gamma))
    os_ = order_statistics(t, np.concatenate([prev, nxt]), device)
    a, b = os_[:prev.size], os_[prev.size:]
    d = b - a  # numpy's _lerp, including its t >= 0.5 branch
    return np.where(gamma >= 0.5, b - d * (1 - gamma), a + d * gamma)


_ = ctypes
