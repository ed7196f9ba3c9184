"""Weight gradient of the narrow 3x3 convolutions (C, Cout multiples of 64, padding 1, stride 1 or 2) on the
hand-written kernel of csrc/conv3_wgrad.hip: one staged input patch per output-row chunk serves all nine taps
(transposed LDS reads, fp32 accumulation, per-split partials summed in order: deterministic).

ResNet-50's stage-1/2 bottleneck 3x3 convolutions (64 and 128 channels) are the users: the grouped split-K GEMM of
mifx.ops.gemm takes the 256+-channel ones and MIOpen's igemm_wrw ran these (profiles/conv3x3_routes_r5.jsonl).
`MIFX_CONV3_WGRAD=0` sends them back to MIOpen (A/B)."""
from __future__ import annotations

import functools
import os

import torch

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle

ENABLED = os.environ.get("MIFX_CONV3_WGRAD", "1") != "0"
# stride 2 measured slower than MIOpen (195-207 vs 147 us, profiles/conv3_wgrad_shapes_r6.jsonl: the 56-wide input
# rows leave room for 3 output rows per chunk, 7 staged input rows for 84 pixels) and a tie in the step: opt-in
_S2 = os.environ.get("MIFX_CONV3_WGRAD_S2", "0") == "1"


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("conv3_wgrad")
    return {"wgrad": sig(lib, "mifx_conv3_wgrad", [VP, VP, VP, VP, I32] + [I32] * 7 + [VP]),
            "splits": sig(lib, "mifx_conv3_wgrad_splits", [I32] * 6),
            "lds": sig(lib, "mifx_conv3_wgrad_lds_bytes", [I32] * 3)}


def eligible(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor, stride: int, route: bool = True) -> bool:
    """x, dy: bf16 channels_last CUDA [N, C, H, W] / [N, Cout, OH, OW]; w: fp32 [Cout, C, 3, 3]. route: also require
    the shapes the kernel is the faster route for (stride 1 unless MIFX_CONV3_WGRAD_S2=1); False: what it supports."""
    if route and stride == 2 and not _S2:
        return False
    if not (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and dy.dtype == torch.bfloat16 and x.dim() == 4
            and stride in (1, 2) and tuple(w.shape[2:]) == (3, 3) and w.dtype == torch.float32
            and x.is_contiguous(memory_format=torch.channels_last)
            and dy.is_contiguous(memory_format=torch.channels_last)
            and (w.is_contiguous() or w.is_contiguous(memory_format=torch.channels_last))):
        return False
    n, c, h, w_ = x.shape
    cout = w.shape[0]
    oh, ow = (h - 1) // stride + 1, (w_ - 1) // stride + 1
    if c % 64 or cout % 64 or w.shape[1] != c or tuple(dy.shape) != (n, cout, oh, ow):
        return False
    return _fns()["lds"](w_, h, stride) > 0


def wgrad(x: torch.Tensor, dy: torch.Tensor, w: torch.Tensor, stride: int) -> torch.Tensor:
    """dW of conv2d(x, w, stride, padding 1) for the upstream gradient dy (eligible() inputs), fp32 in w's layout."""
    n, c, h, w_ = x.shape
    cout = w.shape[0]
    f = _fns()
    splits = f["splits"](n, h, w_, c, cout, stride)
    part = torch.empty(splits * cout * 9 * c, device=x.device, dtype=torch.float32)
    dw = torch.empty_like(w)
    check(f["wgrad"](ptr(x), ptr(dy), ptr(part), ptr(dw), int(not w.is_contiguous()), n, h, w_, c, cout, stride,
                     splits, stream_handle(x.device)), "mifx_conv3_wgrad")
    return dw
