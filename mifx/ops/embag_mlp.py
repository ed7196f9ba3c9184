"""ctypes bindings for csrc/embag_mlp.hip (KFP taxi DNN gather fwd/bwd + sparse Adagrad)."""
from __future__ import annotations

import ctypes
import functools

import torch

from . import _lib
from ._lib import F32, I32, I64, U64, VP, check, ptr, sig, stream_handle


I64 = ctypes.c_longlong


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("embag_mlp")
    return {
        "limits": sig(lib, "mifx_tdnn_limits", [VP]),
        "max_batch": sig(lib, "mifx_tdnn_max_batch", []),
        "fwd_bwd": sig(lib, "mifx_tdnn_fwd_bwd", [VP, VP, VP, VP, VP, I32, VP, I32, I32, VP, I64, VP, I64, I32, I32,
                                                  F32, I32, VP, VP, VP, VP, VP, VP, VP, I64, I64, U64, VP, VP]),
        "adagrad": sig(lib, "mifx_tdnn_adagrad", [VP, VP, VP, VP, VP, VP, VP, VP, VP, I32, VP, I32, I32, I64, VP, I64,
                                                  VP, VP, VP, I32, I32, F32, VP, I64, I64, U64, VP]),
        "chunks": sig(lib, "mifx_tdnn_chunks", [I32]),
    }


def limits() -> dict:
    out = (ctypes.c_int * 3)()
    _fns()["limits"](out)
    return {"max_hidden": out[0], "max_fields": out[1], "max_dense": out[2], "max_batch": _fns()["max_batch"]()}


def make_buffers(B: int, H: int, D: int, device) -> dict:
    """Activation / gradient / scratch buffers for batch B (reused every step)."""
    nh = (H + 255) // 256
    return {"a": torch.empty(B, H, device=device), "dz": torch.empty(B, H, device=device),
            "part": torch.empty(B * nh, device=device), "logit": torch.empty(B, device=device),
            "dlogit": torch.empty(B, device=device), "loss": torch.empty(B, device=device),
            "dpart": torch.empty(_fns()["chunks"](B) * (D + 2) * H, device=device)}


def _feed(feed, B: int) -> tuple[int, int, int]:
    gs, go, key = feed if feed is not None else (B, 0, 0)
    return int(gs), int(go), int(key) & (2**64 - 1)


def fwd_bwd(W1, b1, w2, b2, rows, xd, y, dense_row0: int, grad_scale: float, train: bool, bufs: dict,
            batch: int | None = None, step_ctr: torch.Tensor | None = None, start: int = 0,
            feed: tuple[int, int, int] | None = None, rec_out: torch.Tensor | None = None):
    """rows int32 [n, F] (global W1 rows), xd float [n, D], y float [n]: the resident records (n = batch for one
    batch). With `step_ctr` (int64 device scalar) example b of the step is the record of stream position
    step * stride + offset + b under `feed` = (stride, offset, shuffle seed) (csrc/feed.h, mifx.data.shuffle;
    default (batch, 0, 0): stored order); without it, record (start + b) % n. Fills bufs (a, dz, logit, dlogit,
    loss) for `batch` examples; rec_out (int64 [batch]) receives the record indices."""
    n, F = rows.shape
    B = n if batch is None else int(batch)
    D = xd.shape[1]
    H = W1.shape[1]
    check(_fns()["fwd_bwd"](ptr(W1), ptr(b1), ptr(w2), ptr(b2), ptr(rows), F, ptr(xd), D, dense_row0,
                            ptr(y), n, ptr(step_ctr), int(start), B, H, float(grad_scale), int(train),
                            ptr(bufs["a"]), ptr(bufs["part"]), ptr(bufs.get("dz")), ptr(bufs["logit"]),
                            ptr(bufs.get("dlogit")), ptr(bufs.get("loss")), ptr(bufs.get("dpart") if train else None),
                            *_feed(feed, B), ptr(rec_out), stream_handle(W1.device)),
          "mifx_tdnn_fwd_bwd")


def adagrad(params: dict, accs: dict, rows: torch.Tensor, xd, dense_row0: int, bufs: dict, lr: float,
            batch: int | None = None, step_ctr: torch.Tensor | None = None, start: int = 0,
            feed: tuple[int, int, int] | None = None) -> None:
    """Sparse-row + dense Adagrad (TF semantics) from the buffers of `fwd_bwd` (same record selection); advances
    `step_ctr` by one at the end of the update. No host synchronisation: graph-capturable."""
    n, F = rows.shape
    B = n if batch is None else int(batch)
    H = params["W1"].shape[1]
    check(_fns()["adagrad"](ptr(params["W1"]), ptr(accs["W1"]), ptr(params["b1"]), ptr(accs["b1"]),
                            ptr(params["w2"]), ptr(accs["w2"]), ptr(params["b2"]), ptr(accs["b2"]),
                            ptr(rows), F, ptr(xd), xd.shape[1], dense_row0, n, ptr(step_ctr), int(start),
                            ptr(bufs["a"]), ptr(bufs["dz"]), ptr(bufs["dlogit"]), B, H, float(lr),
                            ptr(bufs["dpart"]), *_feed(feed, B), stream_handle(rows.device)), "mifx_tdnn_adagrad")
