"""3x3 / stride 2 max pooling for NHWC bf16 activations (csrc/pool.hip): 1-byte window argmax, gather-form
deterministic backward. Used by the ResNet-50 stem (pad 1) and the PATE CNN's TF-SAME pooling (teachers and the
teacher ensemble); other shapes / dtypes / layouts run F.max_pool2d."""
from __future__ import annotations

import functools

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("pool")
    return {"fwd": sig(lib, "mifx_maxpool3s2p_fwd", [VP] + [I32] * 9 + [VP, VP, VP]),
            "bwd": sig(lib, "mifx_maxpool3s2p_bwd", [VP, VP] + [I32] * 8 + [VP, VP])}


def native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype == torch.bfloat16 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


def _out_hw(H: int, W: int) -> tuple[int, int]:
    return (H - 1) // 2 + 1, (W - 1) // 2 + 1


class _MaxPool3s2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pt, pl, OH, OW, relu=False):
        N, C, H, W = x.shape
        y = torch.empty((N, C, OH, OW), device=x.device, dtype=x.dtype, memory_format=torch.channels_last)
        idx = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.uint8)
        check(_fns()["fwd"](ptr(x), N, H, W, C, pt, pl, OH, OW, int(relu), ptr(y), ptr(idx), stream_handle(x.device)),
              "mifx_maxpool3s2p_fwd")
        ctx.save_for_backward(idx)
        ctx.shape = (N, C, H, W, pt, pl, OH, OW)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, pt, pl, OH, OW = ctx.shape
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), device=dy.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        check(_fns()["bwd"](ptr(dy), ptr(idx), N, H, W, C, pt, pl, OH, OW, ptr(dx), stream_handle(dy.device)),
              "mifx_maxpool3s2p_bwd")
        return dx, None, None, None, None, None


def max_pool3s2(x: torch.Tensor) -> torch.Tensor:
    """F.max_pool2d(x, 3, 2, 1) -- the HIP kernels for NHWC bf16 on the GPU."""
    if native_ok(x):
        OH, OW = _out_hw(*x.shape[2:])
        return _MaxPool3s2.apply(x, 1, 1, OH, OW)
    return F.max_pool2d(x, 3, 2, 1)


def same_pads(H: int) -> tuple[int, int]:
    """TF 'SAME' 3/2 pooling: output size and top (left) padding."""
    out = -(-H // 2)
    return out, max((out - 1) * 2 + 3 - H, 0) // 2


def max_pool3s2_same(x: torch.Tensor, relu: bool = False) -> torch.Tensor | None:
    """TF-SAME 3x3/2 max pool (padding never wins) of x, or of relu(x) with `relu` (one pass each way: the ReLU's
    backward mask comes free from the window max), on the HIP kernels for NHWC bf16; None when not applicable."""
    if not native_ok(x):
        return None
    (OH, pt), (OW, pl) = same_pads(x.shape[2]), same_pads(x.shape[3])
    return _MaxPool3s2.apply(x, pt, pl, OH, OW, bool(relu))
