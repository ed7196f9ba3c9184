"""Hand-written gfx950 MFMA GEMM (csrc/gemm.hip): Y = X W^T [+ bias] [-> GELU] for nn.Linear-shaped products.

`linear(x, w, bias)` and `linear_bias_gelu(x, w, bias)` are autograd functions whose FORWARD runs the HIP kernel
(with the bias / bias + GELU epilogue fused) and whose backward uses the library GEMMs for dX = dY W and
dW = dY^T X (plus, for GELU, the existing fused bias-GELU backward kernel: the forward saves exactly what
mifx.ops.fused_bert._BiasGelu saves). Shapes the kernel does not tile (M % BM, N % BN, K % 64) take F.linear.

Tile configuration per (M, N, K): the one with the best measured time on MI355X (tools/bench_gemm_hip.py,
profiles/gemm_hip_r3.jsonl) where known, else the heuristic below (fill >= ~1 wave of workgroups on 256 CUs).
"""
from __future__ import annotations

import ctypes
import functools
import os

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("gemm")
    return {
        "configs": sig(lib, "mifx_gemm_configs", [VP, I32]),
        "nt": sig(lib, "mifx_gemm_nt", [I32, I32, I32, VP, VP, VP, VP, VP, I32, I32, I32, VP]),
    }


@functools.lru_cache(maxsize=None)
def configs() -> tuple[tuple[int, int], ...]:
    """(BM, BN) of every compiled tile configuration, by index."""
    return tuple(c[:2] for c in config_details())


@functools.lru_cache(maxsize=None)
def config_details() -> tuple[tuple[int, int, int], ...]:
    """(BM, BN, OPT bits) by index (csrc/gemm.hip kCfgs)."""
    buf = (ctypes.c_int * 96)()
    n = _fns()["configs"](buf, 96)
    return tuple((buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(n))


# Where the hand-written kernel is USED by default (linear / linear_bias_gelu without force=True): the (M, N, K)
# products it measured faster than hipBLASLt on MI355X, with the winning configuration (tools/bench_gemm_hip.py,
# profiles/gemm_hip_r3b.jsonl; BERT-base, 4096 tokens): attention-out 4096x768x768 10.7 us vs 20.5 us. Measured
# slower there and left on hipBLASLt: QKV 22.9 vs 21.6 us, FFN-in 25.3 vs 23.3 us (with the bias + GELU epilogue
# 37.5 vs 34.9 us for GEMM + separate bias_gelu: the epilogue's second 25 MB output (the pre-bias product the
# backward needs) is written after the last K-tile by every workgroup at once, un-overlapped, and a branch-free erf
# did not change that: profiles/gemm_hip_r3c_fasterf.jsonl), FFN-out 28.9 vs 25.1 us. MIFX_HIP_GEMM=all routes every
# eligible shape to the kernel (heuristic configuration) for A/B runs.
TUNED: dict[tuple[int, int, int], int] = {(4096, 768, 768): 13}


def pick_config(M: int, N: int, K: int, cus: int = 256) -> int | None:
    """Index of the tile configuration for an M x N x K product, None if no configuration tiles it."""
    if (M, N, K) in TUNED:
        return TUNED[(M, N, K)]
    best, best_score = None, None
    for i, (bm, bn) in enumerate(configs()):
        if M % bm or N % bn or K % 64:
            continue
        tiles = (M // bm) * (N // bn)
        waves = -(-tiles // cus)
        fill = tiles / (waves * cus)  # useful fraction of the last wave of workgroups
        score = (fill * (bm * bn) ** 0.25, bm * bn)  # prefer full waves, then bigger tiles (operand reuse)
        if best_score is None or score > best_score:
            best, best_score = i, score
    return best


def eligible(x: torch.Tensor, w: torch.Tensor) -> bool:
    """The kernel can compute x @ w^T (bf16 CUDA tensors, a configuration tiles the shape)."""
    if not (x.is_cuda and w.is_cuda and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16):
        return False
    M = x.numel() // x.shape[-1]
    N, K = w.shape
    return x.shape[-1] == K and pick_config(M, N, K) is not None


def preferred(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Eligible AND measured faster than the library for this shape (TUNED), or MIFX_HIP_GEMM=all."""
    if not eligible(x, w):
        return False
    if os.environ.get("MIFX_HIP_GEMM") == "all":
        return True
    return (x.numel() // x.shape[-1], *w.shape) in TUNED


def gemm_nt(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, epi: int = 0,
            cfg: int | None = None) -> tuple[torch.Tensor, torch.Tensor | None]:
    """x2 [M, K] bf16, w [N, K] bf16 -> (Y [M, N] bf16, Z or None). epi 0: X W^T; 1: + bias; 2: GELU(X W^T + bias)
    with Z = bf16(X W^T) (pre-bias)."""
    M, K = x2.shape
    N = w.shape[0]
    if cfg is None:
        cfg = pick_config(M, N, K)
    if cfg is None:
        raise ValueError(f"no GEMM tile configuration for {M}x{N}x{K}")
    x2, w = x2.contiguous(), w.contiguous()
    y = torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    z = torch.empty_like(y) if epi == 2 else None
    b = None
    if epi:
        b = bias if bias.dtype in (torch.float32, torch.bfloat16) else bias.float()
        b = b.contiguous()
    check(_fns()["nt"](int(cfg), int(epi), int(b is not None and b.dtype == torch.float32), ptr(x2), ptr(w), ptr(b),
                       ptr(y), ptr(z), M, N, K, stream_handle(x2.device)), "mifx_gemm_nt")
    return y, z


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y, _ = gemm_nt(x2, w, bias, 1 if bias is not None else 0)
        ctx.save_for_backward(x2, w)
        ctx.has_bias = bias is not None
        ctx.bdtype = bias.dtype if bias is not None else None
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(x2.dtype)
        dx = (dy2 @ w).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        dw = dy2.t() @ x2 if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            from .fused_bert import col_sum

            db = col_sum(dy2, ctx.bdtype if ctx.bdtype in (torch.float32, torch.bfloat16) else torch.float32)
        return dx, dw, db


class _LinearBiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y, z = gemm_nt(x2, w, bias, 2)
        from .fused_bert import _param

        ctx.save_for_backward(x2, w, z, _param(bias))
        ctx.bdtype = bias.dtype
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        from .fused_bert import _dt, _fns as fb_fns

        x2, w, z, bp = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous().to(z.dtype)
        M, N = z.shape
        dz = torch.empty_like(z)
        part = torch.empty(fb_fns()["gchunks"](M), N, device=z.device, dtype=torch.float32)
        db = torch.empty(N, device=z.device, dtype=bp.dtype)
        check(fb_fns()["gelu"](_dt(z), _dt(bp), 0, ptr(dy2), ptr(z), ptr(bp), M, N, ptr(dz), ptr(part), ptr(db),
                               stream_handle(z.device)), "mifx_bert_bias_gelu")
        dx = (dz @ w).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        dw = dz.t() @ x2 if ctx.needs_input_grad[1] else None
        return dx, dw, db if bp.dtype == ctx.bdtype else db.to(ctx.bdtype)


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, force: bool = False) -> torch.Tensor:
    """F.linear with the forward on the hand-written kernel (bias fused) where it is preferred (or, force=True,
    wherever it tiles the shape)."""
    if eligible(x, w) if force else preferred(x, w):
        return _Linear.apply(x, w, bias)
    return F.linear(x, w, bias)


def linear_bias_gelu(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, force: bool = False) -> torch.Tensor:
    """GELU(x w^T + bias) with the bias + GELU fused into the GEMM epilogue where preferred (force: wherever it
    tiles)."""
    if eligible(x, w) if force else preferred(x, w):
        return _LinearBiasGelu.apply(x, w, bias)
    from .fused_bert import bias_gelu

    return bias_gelu(F.linear(x, w), bias)
