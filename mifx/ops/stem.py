"""ResNet-50's stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) on the hand-written MFMA kernels
(csrc/stem_conv.hip): forward and weight gradient (per-workgroup fp32 partials summed in order: deterministic). An
input gradient, which the training step never needs (the stem's input is the preprocessed image), goes to MIOpen.

`stem_conv(x, w)` = F.conv2d(x, w, stride=2, padding=3) for a channels_last bf16 CUDA input of 3 channels (the bf16
forward computes in fp32 from the bf16 image of w, as the autocast path did); elsewhere the PyTorch convolution."""
from __future__ import annotations

import functools
import os

import torch
import torch.nn.functional as F

from . import _lib, native_stats
from ._lib import I32, VP, check, ptr, sig, stream_handle

ENABLED = os.environ.get("MIFX_STEM", "1") != "0"


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("stem_conv")
    return {"fwd": sig(lib, "mifx_stem_fwd", [VP, VP, I32, VP, VP, I32, I32, I32, VP]),
            "wgrad": sig(lib, "mifx_stem_wgrad", [VP, VP, VP, VP, I32, I32, I32, I32, VP]),
            "splits": sig(lib, "mifx_stem_wgrad_splits", [I32])}


# MIFX_STEM_WGRAD=0: the weight gradient on MIOpen (A/B)
_WGRAD = os.environ.get("MIFX_STEM_WGRAD", "1") != "0"


def eligible(x: torch.Tensor, w: torch.Tensor) -> bool:
    return (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] == 3
            and x.is_contiguous(memory_format=torch.channels_last) and tuple(w.shape) == (64, 3, 7, 7)
            and w.dtype == torch.float32 and w.is_cuda
            and (w.is_contiguous() or w.is_contiguous(memory_format=torch.channels_last)))


class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        n, _, h, wd = x.shape
        oh, ow = (h - 1) // 2 + 1, (wd - 1) // 2 + 1
        y = torch.empty(n, 64, oh, ow, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        img = torch.empty(64 * 7 * 32, device=x.device, dtype=torch.bfloat16)
        cl = int(not w.is_contiguous())
        check(_fns()["fwd"](ptr(x), ptr(w), cl, ptr(img), ptr(y), n, h, wd, stream_handle(x.device)), "mifx_stem_fwd")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dx = dw = None
        if ctx.needs_input_grad[1] and _WGRAD:
            n, _, h, wd = x.shape
            part = torch.empty(n * _fns()["splits"](n) * 64 * 7 * 32, device=x.device, dtype=torch.float32)
            dw = torch.empty_like(w)  # (same layout as the parameter: the kernel writes either)
            check(_fns()["wgrad"](ptr(x), ptr(dy), ptr(part), ptr(dw), int(not w.is_contiguous()), n, h, wd,
                                  stream_handle(x.device)), "mifx_stem_wgrad")
        if ctx.needs_input_grad[0] or (ctx.needs_input_grad[1] and dw is None):
            wb = w.to(torch.bfloat16)
            dx, dwm, _ = torch.ops.aten.convolution_backward(
                dy, x, wb, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                [ctx.needs_input_grad[0], ctx.needs_input_grad[1] and dw is None, False])
            if dw is None and dwm is not None:
                dw = dwm.to(w.dtype)
        return dx, dw


def stem_conv(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """conv2d(x, w, stride 2, padding 3) -- the hand-written forward where eligible()."""
    if eligible(x, w):
        native_stats.count("stem_fwd", True)
        return _Stem.apply(x, w)
    if x.is_cuda:
        native_stats.count("stem_fwd", False)
    return F.conv2d(x, w.to(x.dtype) if x.is_cuda else w, None, 2, 3)
