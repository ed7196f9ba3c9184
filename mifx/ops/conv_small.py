"""Direct fp32 convolutions for the reference's small MNIST / Fashion-MNIST CNNs (csrc/conv_small.hip).

`SmallConv2d` is an nn.Conv2d whose CUDA fp32 forward AND backward run the hand-written kernels (no MIOpen); on the
CPU, or for shapes outside the kernels' envelope (R * S > 64, groups, dilation), it is plain nn.Conv2d. `same=True`
reproduces TF "SAME" padding (asymmetric when needed) by splitting it into the symmetric part the kernels take and an
explicit one-sided pad.
"""
from __future__ import annotations

import functools
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle

# Input channels up to which the VALU direct conv is used: the first layers (1 or 3 channels) of these CNNs, where
# an MFMA tile has nothing to reduce over. Per model by measurement (tools/bench_cnn.py,
# profiles/archive/cnn_small_conv_r3.jsonl): MIOpen is faster on all but the Fashion CNN -- TPU CNN 1.46 ms/step with its
# first layer direct (6.8 with every layer direct) vs 1.29, DP-SGD tutorial SGD step 0.67 vs 0.60, PATE teacher 1.75
# vs 1.60; Fashion 0.43-0.49 vs 0.54, so FashionCNN's conv runs here by default (prefer=True) and the others only
# with MIFX_SMALL_CONV=1 (MIFX_SMALL_CONV=0 turns every direct conv off).
MAX_CIN = 4
MAX_WEIGHTS = 40_000


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("conv_small")
    a = [VP, VP, VP, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, I32, VP]
    return {"fwd": sig(lib, "mifx_convs_fwd", [VP] + a),
            "dgrad": sig(lib, "mifx_convs_dgrad", a),
            "wgrad": sig(lib, "mifx_convs_wgrad", [VP] + a),
            "splits": sig(lib, "mifx_convs_wgrad_splits", [I32, I32, I32, I32, I32])}


def _in_functorch_transform() -> bool:
    """Inside vmap / grad (the DP-SGD per-example fallback): a plain autograd.Function cannot be transformed."""
    try:
        return torch._C._functorch.peek_interpreter_stack() is not None
    except AttributeError:  # pragma: no cover - older torch
        return False


def eligible(x: torch.Tensor, w: torch.Tensor, groups: int = 1, dilation=(1, 1), prefer: bool = False) -> bool:
    """MIFX_SMALL_CONV=1 turns the direct kernels on (default: library convolutions, measured faster), =0 off;
    unset: on only for layers whose model measured faster on them (prefer=True)."""
    env = os.environ.get("MIFX_SMALL_CONV")
    on = env == "1" if env is not None else prefer
    return (on and x.is_cuda and x.dtype == torch.float32
            and w.dtype == torch.float32 and x.dim() == 4 and groups == 1 and tuple(dilation) == (1, 1)
            and w.shape[1] <= MAX_CIN and w.shape[2] * w.shape[3] <= 64 and w.numel() <= MAX_WEIGHTS
            and not _in_functorch_transform())


def _geo(x, w, stride, ph, pw):
    N, C, H, W = x.shape
    K, _, R, S = w.shape
    Ho, Wo = (H + 2 * ph - R) // stride + 1, (W + 2 * pw - S) // stride + 1
    return N, C, H, W, K, R, S, stride, ph, pw, Ho, Wo


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, ph, pw):
        x, w = x.contiguous(), w.contiguous()
        g = _geo(x, w, stride, ph, pw)
        y = torch.empty(g[0], g[4], g[10], g[11], device=x.device, dtype=torch.float32)
        bb = b.contiguous() if b is not None else None
        check(_fns()["fwd"](ptr(x), ptr(w), ptr(bb), ptr(y), *g, stream_handle(x.device)), "mifx_convs_fwd")
        ctx.save_for_backward(x, w)
        ctx.g, ctx.has_b = g, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous().float()
        dx = dw = db = None
        s = stream_handle(x.device)
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            check(_fns()["dgrad"](ptr(dy), ptr(w), ptr(dx), *ctx.g, s), "mifx_convs_dgrad")
        if ctx.needs_input_grad[1]:
            dw = torch.empty_like(w)
            N, C, _, _, K, R, S, _, _, _, Ho, Wo = ctx.g
            part = torch.empty(_fns()["splits"](N, K, C, Ho, Wo) * w.numel(), device=w.device)
            check(_fns()["wgrad"](ptr(x), ptr(dy), ptr(dw), ptr(part), *ctx.g, s), "mifx_convs_wgrad")
        if ctx.has_b and ctx.needs_input_grad[2]:
            db = dy.sum((0, 2, 3))
        return dx, dw, db, None, None, None


def conv2d(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, stride: int = 1, padding: int = 0):
    """Symmetric-padding fp32 NCHW convolution on the direct kernels."""
    return _Conv.apply(x, w, b, int(stride), int(padding), int(padding))


def same_split(h: int, w: int, k: int, s: int) -> tuple[int, int, tuple[int, int, int, int]]:
    """TF SAME padding as (symmetric pad_h, symmetric pad_w, extra F.pad (left, right, top, bottom))."""
    ph = max((math.ceil(h / s) - 1) * s + k - h, 0)
    pw = max((math.ceil(w / s) - 1) * s + k - w, 0)
    return ph // 2, pw // 2, (0, pw - 2 * (pw // 2), 0, ph - 2 * (ph // 2))


class SmallConv2d(nn.Conv2d):
    """nn.Conv2d (stride s, symmetric `padding`, or TF SAME with same=True) on the direct HIP kernels for CUDA fp32."""

    def __init__(self, cin, cout, k, stride=1, padding=0, same: bool = False, prefer: bool = False):
        super().__init__(cin, cout, k, stride=stride, padding=0 if same else padding)
        self.same = same
        self.prefer = prefer  # the model measured faster with this layer on the direct kernels (default on)

    def forward(self, x):
        s = self.stride[0]
        if not (eligible(x, self.weight, self.groups, self.dilation, self.prefer) and self.stride[0] == self.stride[1]):
            if self.same:  # the library path exactly as before: explicit SAME pad, unpadded conv
                ph, pw, extra = same_split(x.shape[-2], x.shape[-1], self.kernel_size[0], s)
                x = F.pad(x, (pw, pw + extra[1], ph, ph + extra[3]))
            return F.conv2d(x, self.weight, self.bias, self.stride, 0 if self.same else self.padding)
        if self.same:
            ph, pw, extra = same_split(x.shape[-2], x.shape[-1], self.kernel_size[0], s)
            if any(extra):
                x = F.pad(x, extra)
        else:
            ph, pw = self.padding
        return _Conv.apply(x, self.weight, self.bias, s, ph, pw)
