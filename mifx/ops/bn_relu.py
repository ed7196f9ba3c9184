"""Fused BatchNorm + ReLU over channels_last activations (csrc/bn_relu.hip).

`BatchNormReLU2d` is a drop-in `nn.BatchNorm2d` (same parameters, buffers and state_dict keys)
whose forward is relu(batch_norm(x)). On the GPU with a channels_last (NHWC) bf16/fp32 input and
C % 8 == 0 it runs the native kernels — training: stats -> finalize (running stats updated on the
device) -> apply; backward: reduce -> finalize -> apply — and fails loudly if the library is
missing. Elsewhere (CPU, other layouts) it runs the PyTorch reference of the same math."""
from __future__ import annotations

import functools

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("bn_relu")
    return {
        "blocks": sig(lib, "mifx_bn_blocks", [I64, I32]),
        "fwd": sig(lib, "mifx_bn_relu_fwd", [I32, VP, I64, I32, VP, VP, F32, F32, VP, VP, I32, VP, VP, VP, VP]),
        "apply": sig(lib, "mifx_bn_relu_apply", [I32, VP, I64, I32, VP, VP, I32, VP, VP]),
        "bwd": sig(lib, "mifx_bn_relu_bwd", [I32, VP, VP, I64, I32, VP, VP, I32, VP, VP, VP, VP, VP, VP]),
    }


def _nhwc_view(x: torch.Tensor) -> torch.Tensor | None:
    """[N, C, H, W] channels_last (or [M, C] row-major) -> the [M, C] storage view, else None."""
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        n, c, h, w = x.shape
        return x.permute(0, 2, 3, 1).reshape(n * h * w, c)
    if x.dim() == 2 and x.is_contiguous():
        return x
    return None


def native_ok(x: torch.Tensor) -> bool:
    if not x.is_cuda or x.dtype not in (torch.bfloat16, torch.float32):
        return False
    v = _nhwc_view(x)
    c = x.shape[1]
    return v is not None and c % 8 == 0 and c <= 2048 and x.data_ptr() % 16 == 0 and v.shape[0] > 0


def _dt(t: torch.Tensor) -> int:
    return 1 if t.dtype == torch.bfloat16 else 0


class _BNReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, run_mean, run_var, momentum, eps, relu):
        v = _nhwc_view(x)
        M, C = v.shape
        w32, b32 = weight.float().contiguous(), bias.float().contiguous()
        nb = _fns()["blocks"](M, C)
        part = torch.empty(2, nb, C, device=x.device, dtype=torch.float32)
        stats = torch.empty(4, C, device=x.device, dtype=torch.float32)
        y = torch.empty_like(x)  # same (channels_last) layout
        rm = run_mean if run_mean is not None else None
        check(_fns()["fwd"](_dt(x), ptr(v), M, C, ptr(w32), ptr(b32), float(eps), float(momentum), ptr(rm),
                            ptr(run_var if rm is not None else None), int(relu), ptr(part), ptr(stats), ptr(y),
                            stream_handle(x.device)), "mifx_bn_relu_fwd")
        ctx.save_for_backward(x, w32, stats)
        ctx.relu, ctx.wdtype = relu, weight.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32, stats = ctx.saved_tensors
        if not dy.is_contiguous(memory_format=torch.channels_last) and dy.dim() == 4:
            dy = dy.contiguous(memory_format=torch.channels_last)
        dy = dy.to(x.dtype)
        v, dv = _nhwc_view(x), _nhwc_view(dy)
        M, C = v.shape
        nb = _fns()["blocks"](M, C)
        part = torch.empty(2, nb, C, device=x.device, dtype=torch.float32)
        kbuf = torch.empty(3, C, device=x.device, dtype=torch.float32)
        dgb = torch.empty(2, C, device=x.device, dtype=torch.float32)
        dx = torch.empty_like(x)
        check(_fns()["bwd"](_dt(x), ptr(dv), ptr(v), M, C, ptr(w32), ptr(stats), int(ctx.relu), ptr(part), ptr(kbuf),
                            ptr(dx), ptr(dgb[0]), ptr(dgb[1]), stream_handle(x.device)), "mifx_bn_relu_bwd")
        return dx, dgb[0].to(ctx.wdtype), dgb[1].to(ctx.wdtype), None, None, None, None, None


def bn_relu(x, weight, bias, running_mean=None, running_var=None, training=True, momentum=0.1, eps=1e-5,
            relu=True):
    """relu(batch_norm(x)) (relu optional). Native on channels_last GPU tensors."""
    if native_ok(x):
        if training:
            return _BNReLU.apply(x, weight, bias, running_mean, running_var, momentum, eps, relu)
        scale = (weight.float() * torch.rsqrt(running_var.float() + eps)).contiguous()
        shift = (bias.float() - running_mean.float() * scale).contiguous()
        v = _nhwc_view(x)
        y = torch.empty_like(x)
        check(_fns()["apply"](_dt(x), ptr(v), v.shape[0], v.shape[1], ptr(scale), ptr(shift), int(relu), ptr(y),
                              stream_handle(x.device)), "mifx_bn_relu_apply")
        return y
    if x.is_cuda and _lib.gpu_available() and x.dim() == 4 and x.shape[1] % 8 == 0 \
            and x.is_contiguous(memory_format=torch.channels_last):
        _fns()  # channels_last GPU input that should have been native: fail loudly if the library is absent
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum, eps)
    return F.relu(y) if relu else y


class BatchNormReLU2d(nn.BatchNorm2d):
    """nn.BatchNorm2d followed by ReLU, fused on the GPU. Parameters/buffers/state_dict == BatchNorm2d."""

    def forward(self, x):
        if self.training and self.track_running_stats:
            self.num_batches_tracked.add_(1)
        use_batch_stats = self.training or not self.track_running_stats
        return bn_relu(x, self.weight, self.bias, self.running_mean if self.track_running_stats else None,
                       self.running_var if self.track_running_stats else None, use_batch_stats, self.momentum,
                       self.eps, True)
