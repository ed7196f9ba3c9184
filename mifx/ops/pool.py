"""3x3 / stride 2 / pad 1 max pooling for NHWC bf16 activations (csrc/pool.hip): 1-byte window argmax,
gather-form deterministic backward. Used by the ResNet-50 stem; other shapes / dtypes / layouts run
F.max_pool2d."""
from __future__ import annotations

import functools

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("pool")
    return {"fwd": sig(lib, "mifx_maxpool3s2_fwd", [VP, I32, I32, I32, I32, VP, VP, VP]),
            "bwd": sig(lib, "mifx_maxpool3s2_bwd", [VP, VP, I32, I32, I32, I32, VP, VP])}


def native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


def _out_hw(H: int, W: int) -> tuple[int, int]:
    return (H - 1) // 2 + 1, (W - 1) // 2 + 1


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        OH, OW = _out_hw(H, W)
        y = torch.empty((N, C, OH, OW), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        idx = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.uint8)
        check(_fns()["fwd"](ptr(x), N, H, W, C, ptr(y), ptr(idx), stream_handle(x.device)), "mifx_maxpool3s2_fwd")
        ctx.save_for_backward(idx)
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W = ctx.shape
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), device=dy.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        check(_fns()["bwd"](ptr(dy), ptr(idx), N, H, W, C, ptr(dx), stream_handle(dy.device)), "mifx_maxpool3s2_bwd")
        return dx


def max_pool3s2(x: torch.Tensor) -> torch.Tensor:
    """F.max_pool2d(x, 3, 2, 1) -- the HIP kernels for NHWC bf16 on the GPU."""
    if native_ok(x):
        return _MaxPool3s2.apply(x)
    return F.max_pool2d(x, 3, 2, 1)
