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
    }


def column_moments(x, device=None) -> dict:
    a = np.asarray(x, dtype=np.float64)
    if not _is_gpu(device):
        v = a[~np.isnan(a)]
        if v.size == 0:
            return {"count": 0, "mean": 0.0, "std": 0.0, "min": 0.0, "max": 0.0, "zeros": 0}
        return {"count": int(v.size), "mean": float(v.mean()), "std": float(v.std()), "min": float(v.min()),
                "max": float(v.max()), "zeros": int((v == 0).sum())}
    dev = torch.device(device)
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    grid = int(max(1, min(1024, (a.size + 255) // 256)))
    part = torch.empty(grid * _fns()["mbytes"](), dtype=torch.uint8, device=dev)
    out = torch.empty(6, dtype=torch.float64, device=dev)
    check(_fns()["moments"](ptr(t), a.size, ptr(part), grid, ptr(out), stream_handle(dev)), "mifx_an_moments")
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


_ = ctypes
