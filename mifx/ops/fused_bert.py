"""Fused residual-add + LayerNorm and bias + GELU (csrc/fused_bert.hip) as autograd functions.

On CUDA/HIP tensors the native kernels run (required — no silent fallback); on CPU the PyTorch
reference implementation of the same math runs."""
from __future__ import annotations

import functools
import os

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("fused_bert")
    return {
        "blocks": sig(lib, "mifx_bert_ln_blocks", [I32]),
        "gchunks": sig(lib, "mifx_bert_gelu_chunks", [I32]),
        "ln_fwd": sig(lib, "mifx_bert_add_ln_fwd", [I32, VP, VP, VP, VP, I32, I32, F32, VP, VP, VP, VP]),
        "ln_bwd": sig(lib, "mifx_bert_add_ln_bwd", [I32, VP, VP, VP, VP, VP, VP, I32, I32, VP, VP, VP, VP, VP, VP]),
        "gelu": sig(lib, "mifx_bert_bias_gelu", [I32, I32, VP, VP, VP, I32, I32, VP, VP, VP, VP]),
    }


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"unsupported dtype {t.dtype}")


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, r, w, b, eps):
        a, r = a.contiguous(), r.contiguous().to(a.dtype)
        H = a.shape[-1]
        R = a.numel() // H
        w32, b32 = w.float().contiguous(), b.float().contiguous()
        y = torch.empty_like(a)
        mean = torch.empty(R, device=a.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        check(_fns()["ln_fwd"](_dt(a), ptr(a), ptr(r), ptr(w32), ptr(b32), R, H, float(eps), ptr(y), ptr(mean),
                               ptr(rstd), stream_handle(a.device)), "mifx_bert_add_ln_fwd")
        ctx.save_for_backward(a, r, w32, mean, rstd)
        ctx.wdtype = w.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        a, r, w32, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous().to(a.dtype)
        H = a.shape[-1]
        R = a.numel() // H
        nb = _fns()["blocks"](R)
        dx = torch.empty_like(a)
        part = torch.empty(2, nb, H, device=a.device, dtype=torch.float32)
        dwdb = torch.empty(2, H, device=a.device, dtype=torch.float32)
        check(_fns()["ln_bwd"](_dt(a), ptr(dy), ptr(a), ptr(r), ptr(w32), ptr(mean), ptr(rstd), R, H, ptr(dx),
                               ptr(part[0]), ptr(part[1]), ptr(dwdb[0]), ptr(dwdb[1]), stream_handle(a.device)),
              "mifx_bert_add_ln_bwd")
        return dx, dx, dwdb[0].to(ctx.wdtype), dwdb[1].to(ctx.wdtype), None


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        x = x.contiguous()
        b32 = bias.float().contiguous()
        y = torch.empty_like(x)
        N = x.shape[-1]
        check(_fns()["gelu"](_dt(x), 1, None, ptr(x), ptr(b32), x.numel() // N, N, ptr(y), None, None,
                             stream_handle(x.device)), "mifx_bert_bias_gelu")
        ctx.save_for_backward(x, b32)
        ctx.bdtype = bias.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, b32 = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        dx = torch.empty_like(x)
        N = x.shape[-1]
        M = x.numel() // N
        part = torch.empty(_fns()["gchunks"](M), N, device=x.device, dtype=torch.float32)
        db = torch.empty(N, device=x.device, dtype=torch.float32)
        check(_fns()["gelu"](_dt(x), 0, ptr(dy), ptr(x), ptr(b32), M, N, ptr(dx), ptr(part), ptr(db),
                             stream_handle(x.device)), "mifx_bert_bias_gelu")
        return dx, db.to(ctx.bdtype)


# diagnostic switch: MIFX_BERT_TORCH_OPS=1 runs the PyTorch reference ops on the GPU too (bisection only)
_TORCH_OPS = os.environ.get("MIFX_BERT_TORCH_OPS") == "1"


def add_layernorm(a: torch.Tensor, r: torch.Tensor, weight, bias, eps: float = 1e-12) -> torch.Tensor:
    """LayerNorm(a + r) * weight + bias."""
    if a.is_cuda and not _TORCH_OPS:
        return _AddLayerNorm.apply(a, r, weight, bias, eps)
    return F.layer_norm(a + r, (a.shape[-1],), weight, bias, eps)


def bias_gelu(x: torch.Tensor, bias) -> torch.Tensor:
    """GELU(erf)(x + bias)."""
    if x.is_cuda and not _TORCH_OPS:
        return _BiasGelu.apply(x, bias)
    return F.gelu(x + bias)
