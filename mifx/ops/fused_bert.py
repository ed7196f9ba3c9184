"""Fused [bias +] [dropout +] residual-add + LayerNorm, standalone dropout and bias + GELU
(csrc/fused_bert.hip) as autograd functions.

On CUDA/HIP tensors the native kernels run (required — no silent fallback); on CPU the PyTorch
reference implementation of the same math runs."""
from __future__ import annotations

import functools
import os

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib
from ._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("fused_bert")
    return {
        "blocks": sig(lib, "mifx_bert_ln_blocks", [I32]),
        "gchunks": sig(lib, "mifx_bert_gelu_chunks", [I32]),
        "ln_fwd": sig(lib, "mifx_bert_bdaln_fwd", [I32, I32, VP, VP, VP, VP, VP, I32, I32, F32, F32, VP, I32, VP, VP,
                                                   VP, VP]),
        "ln_bwd": sig(lib, "mifx_bert_bdaln_bwd", [I32, I32, VP, VP, VP, VP, VP, VP, VP, I32, I32, F32, VP, I32, VP,
                                                   VP, VP, VP, VP, VP, VP]),
        "ln_fwd2": sig(lib, "mifx_bert_bdaln_fwd2", [I32, I32, VP, VP, VP, VP, VP, I32, I32, F32, F32, VP, I32, I64,
                                                     VP, VP, VP, VP]),
        "ln_bwd2": sig(lib, "mifx_bert_bdaln_bwd2", [I32, I32, VP, VP, VP, VP, VP, VP, VP, I32, I32, F32, VP, I32, I64,
                                                     VP, VP, VP, VP, VP, VP, VP]),
        "dropout": sig(lib, "mifx_bert_dropout", [I32, VP, I64, F32, VP, I32, VP, VP]),
        "gelu": sig(lib, "mifx_bert_bias_gelu", [I32, I32, I32, VP, VP, VP, I32, I32, VP, VP, VP, VP]),
        "colsum": sig(lib, "mifx_bert_col_sum", [I32, I32, VP, I32, I32, VP, VP, VP]),
        "emb_bwd": sig(lib, "mifx_bert_emb_bwd", [I32, VP, I32, VP, I32, I64, VP, I32, VP, VP, VP]),
    }


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 1
    if t.dtype == torch.float32:
        return 0
    raise TypeError(f"unsupported dtype {t.dtype}")


def _param(p: torch.Tensor) -> torch.Tensor:
    """LayerNorm / bias parameters are read in their own dtype (fp32 or bf16) by the kernels."""
    p = p if p.dtype in (torch.float32, torch.bfloat16) else p.float()
    return p.contiguous()


# ---- counter-based dropout masks (same bits as the HIP kernels in csrc/fused_bert.hip)
_M64 = (1 << 64) - 1
_GOLDEN = 0x9E3779B97F4A7C15


def _mix64(z: np.ndarray) -> np.ndarray:
    """murmur3 fmix64 on a uint64 array (wrapping arithmetic)."""
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xFF51AFD7ED558CCD)
    z = z ^ (z >> np.uint64(33))
    z = z * np.uint64(0xC4CEB9FE1A85EC53)
    return z ^ (z >> np.uint64(33))


def drop_threshold(p: float) -> int:
    """keep element iff its 16-bit hash lane >= threshold (float32 math, as the kernel computes it)."""
    if not p > 0:
        return 0
    t = np.float32(p) * np.float32(65536.0) + np.float32(0.5)
    return 65536 if t >= 65536 else int(t)


def keep_mask(n: int, rng: torch.Tensor, site: int, p: float) -> torch.Tensor:
    """Bool keep-mask of n flat elements for (rng = [seed, counter], site): the host twin of the kernels'
    keep4(drop_key(rng, site), g, thr) — group g of 4 consecutive elements takes the four 16-bit lanes of
    mix64(key + g * golden)."""
    seed, ctr = (int(v) for v in rng.detach().cpu().tolist()[:2])
    with np.errstate(over="ignore"):
        inner = _mix64(np.array([(ctr * _GOLDEN + site) & _M64], dtype=np.uint64))
        key = _mix64(np.array([seed & _M64], dtype=np.uint64) ^ inner)
        g = np.arange((n + 3) // 4, dtype=np.uint64)
        h = _mix64(key + g * np.uint64(_GOLDEN))
    lanes = (h[:, None] >> np.array([0, 16, 32, 48], dtype=np.uint64)) & np.uint64(0xFFFF)
    keep = (lanes >= np.uint64(drop_threshold(p))).reshape(-1)[:n]
    return torch.from_numpy(keep)


def rng_snapshot(rng: torch.Tensor) -> torch.Tensor:
    """A frozen copy of the [seed, counter] state for one model forward: every dropout site of that forward reads it
    (forward and recomputed-mask backward), so no site needs its own copy. One device copy per forward instead of
    one per site (each a ~4.6 us copy node in the captured BERT step: 45 per step)."""
    snap = rng.detach().clone()
    snap._mifx_frozen = True
    return snap


def _snap(rng, p) -> torch.Tensor | None:
    """The dropout RNG state as it is when the forward runs (None without dropout): the tensor itself when it is a
    frozen per-forward snapshot (rng_snapshot), else a device copy (the live counter may advance before the
    backward: two training forwards before one backward, activation checkpointing)."""
    if rng is None or p <= 0:
        return None
    return rng if getattr(rng, "_mifx_frozen", False) else rng.detach().clone()


def device_keep_mask(n: int, rng: torch.Tensor, site: int, p: float, device) -> torch.Tensor:
    """keep_mask computed on the GPU (no host sync; graph-capturable): the dropout kernel applied to ones."""
    ones = torch.ones(n, device=device, dtype=torch.float32)
    y = torch.empty_like(ones)
    check(_fns()["dropout"](_dt(ones), ptr(ones), n, float(p), ptr(rng), int(site), ptr(y), stream_handle(device)),
          "mifx_bert_dropout(mask)")
    return y != 0


def _mask(n: int, rng, site: int, p: float, device) -> torch.Tensor:
    if torch.device(device).type == "cuda" and rng is not None and rng.is_cuda and not _TORCH_OPS:
        return device_keep_mask(n, rng, site, p, device)
    return keep_mask(n, rng, site, p).to(device)


def _drop_scale(p: float) -> float:
    return float(np.float32(1.0) / (np.float32(1.0) - np.float32(p)))


class _BiasDropAddLN(torch.autograd.Function):
    """y = LayerNorm(dropout_p(a [+ bias]) + r) * w + b in one HIP kernel (and one backward kernel producing
    dr, da and the gamma / beta / bias gradients); the dropout mask is recomputed in the backward."""

    @staticmethod
    def forward(ctx, a, bias, r, w, b, eps, p, rng, site, slot=None, eoff=0):
        a, r = a.contiguous(), r.contiguous().to(a.dtype)
        H = a.shape[-1]
        R = a.numel() // H
        wp = _param(w)
        bp = _param(b.to(wp.dtype))
        biasp = None if bias is None else _param(bias.to(wp.dtype))
        y = torch.empty_like(a)
        mean = torch.empty(R, device=a.device, dtype=torch.float32)
        rstd = torch.empty_like(mean)
        check(_fns()["ln_fwd2"](_dt(a), _dt(wp), ptr(a), ptr(biasp), ptr(r), ptr(wp), ptr(bp), R, H, float(eps),
                                float(p), ptr(rng if p > 0 else None), int(site), int(eoff), ptr(y), ptr(mean),
                                ptr(rstd), stream_handle(a.device)), "mifx_bert_bdaln_fwd")
        ctx.save_for_backward(a, r, wp, biasp, mean, rstd)
        # snapshot of [seed, counter] at forward time (a device copy, graph-capturable): the backward recomputes
        # the forward's mask even if the live counter advanced in between (activation re-forward, 2 forwards)
        ctx.rng, ctx.p, ctx.site, ctx.eoff = _snap(rng, p), float(p), int(site), int(eoff)
        ctx.wdtype = w.dtype
        ctx.bdtype = None if bias is None else bias.dtype
        ctx.slot = slot
        return y

    @staticmethod
    def backward(ctx, dy):
        a, r, wp, biasp, mean, rstd = ctx.saved_tensors
        dy = dy.contiguous().to(a.dtype)
        H = a.shape[-1]
        R = a.numel() // H
        nb = _fns()["blocks"](R)
        dr = torch.empty_like(a)
        da = torch.empty_like(a) if (ctx.p > 0 or biasp is not None) else dr
        part = torch.empty(3, nb, H, device=a.device, dtype=torch.float32)
        dw = torch.empty(H, device=a.device, dtype=wp.dtype)  # written in the parameter dtype by the kernel
        db = torch.empty(H, device=a.device, dtype=wp.dtype)
        dbias = None if biasp is None else torch.empty(H, device=a.device, dtype=wp.dtype)
        check(_fns()["ln_bwd2"](_dt(a), _dt(wp), ptr(dy), ptr(a), ptr(biasp), ptr(r), ptr(wp), ptr(mean), ptr(rstd),
                                R, H, ctx.p, ptr(ctx.rng if ctx.p > 0 else None), ctx.site, ctx.eoff, ptr(dr), ptr(da),
                                ptr(part), ptr(dw), ptr(db), ptr(dbias), stream_handle(a.device)),
              "mifx_bert_bdaln_bwd")
        if wp.dtype != ctx.wdtype:
            dw, db = dw.to(ctx.wdtype), db.to(ctx.wdtype)
        if dbias is not None and dbias.dtype != ctx.bdtype:
            dbias = dbias.to(ctx.bdtype)
        if ctx.slot is not None:  # the residual's other consumer folds dr into its input-gradient GEMM
            ctx.slot.g, dr = dr, None
        return da, dbias, dr, dw, db, None, None, None, None, None, None


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, rng, site):
        x = x.contiguous()
        y = torch.empty_like(x)
        check(_fns()["dropout"](_dt(x), ptr(x), x.numel(), float(p), ptr(rng), int(site), ptr(y),
                                stream_handle(x.device)), "mifx_bert_dropout")
        ctx.rng, ctx.p, ctx.site = _snap(rng, p), float(p), int(site)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        check(_fns()["dropout"](_dt(dy), ptr(dy), dy.numel(), ctx.p, ptr(ctx.rng), ctx.site, ptr(dx),
                                stream_handle(dy.device)), "mifx_bert_dropout")
        return dx, None, None, None


class _BiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias):
        x = x.contiguous()
        bp = _param(bias)
        y = torch.empty_like(x)
        N = x.shape[-1]
        check(_fns()["gelu"](_dt(x), _dt(bp), 1, None, ptr(x), ptr(bp), x.numel() // N, N, ptr(y), None, None,
                             stream_handle(x.device)), "mifx_bert_bias_gelu")
        ctx.save_for_backward(x, bp)
        ctx.bdtype = bias.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        x, bp = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        dx = torch.empty_like(x)
        N = x.shape[-1]
        M = x.numel() // N
        part = torch.empty(_fns()["gchunks"](M), N, device=x.device, dtype=torch.float32)
        db = torch.empty(N, device=x.device, dtype=bp.dtype)  # written in the bias dtype by the kernel
        check(_fns()["gelu"](_dt(x), _dt(bp), 0, ptr(dy), ptr(x), ptr(bp), M, N, ptr(dx), ptr(part), ptr(db),
                             stream_handle(x.device)), "mifx_bert_bias_gelu")
        return dx, db if bp.dtype == ctx.bdtype else db.to(ctx.bdtype)


def col_sum(x: torch.Tensor, out_dtype: torch.dtype) -> torch.Tensor:
    """Column sums of a 2-D [M, N] fp32/bf16 tensor -> [N] in out_dtype (fp32 or bf16): the bias gradient,
    deterministic (fixed-order partials + col_reduce2) instead of a generic reduction kernel."""
    x = x.contiguous()
    M, N = x.shape
    if not x.is_cuda or _TORCH_OPS:
        return x.float().sum(0).to(out_dtype)
    pdt = out_dtype if out_dtype in (torch.float32, torch.bfloat16) else torch.float32
    part = torch.empty(_fns()["gchunks"](M), N, device=x.device, dtype=torch.float32)
    out = torch.empty(N, device=x.device, dtype=pdt)
    check(_fns()["colsum"](_dt(x), int(pdt == torch.bfloat16), ptr(x), M, N, ptr(part), ptr(out),
                           stream_handle(x.device)), "mifx_bert_col_sum")
    return out if pdt == out_dtype else out.to(out_dtype)


def _compute_dtype(x: torch.Tensor) -> torch.dtype:
    if x.is_cuda and torch.is_autocast_enabled("cuda"):
        return torch.get_autocast_dtype("cuda")
    return x.dtype


class _BiasAdd(torch.autograd.Function):
    """y + bias (broadcast over leading dims); backward: bias grad by col_sum."""

    @staticmethod
    def forward(ctx, y, bias):
        ctx.bdtype = bias.dtype
        return y + bias.to(y.dtype)

    @staticmethod
    def backward(ctx, dy):
        return dy, col_sum(dy.reshape(-1, dy.shape[-1]), ctx.bdtype)


class _Linear(torch.autograd.Function):
    """F.linear(x, w, b) (bias in the GEMM epilogue) with the backward's bias gradient by col_sum; casts
    to the autocast dtype itself (like F.linear under autocast) and returns gradients in the inputs' dtypes."""

    @staticmethod
    def forward(ctx, x, w, b):
        cdt = _compute_dtype(x)
        with torch.autocast("cuda", enabled=False):
            xc, wc = x.to(cdt), w.to(cdt)
            y = F.linear(xc, wc, None if b is None else b.to(cdt))
        ctx.save_for_backward(xc, wc)
        ctx.dtypes = (x.dtype, w.dtype, None if b is None else b.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xc, wc = ctx.saved_tensors
        xdt, wdt, bdt = ctx.dtypes
        with torch.autocast("cuda", enabled=False):
            dy = dy.to(wc.dtype)
            dy2 = dy.reshape(-1, dy.shape[-1])
            dx = dw = db = None
            if ctx.needs_input_grad[0]:
                dx = dy.matmul(wc).to(xdt)
            if ctx.needs_input_grad[1]:
                dw = dy2.t().mm(xc.reshape(-1, xc.shape[-1])).to(wdt)
            if bdt is not None and ctx.needs_input_grad[2]:
                db = col_sum(dy2, bdt)
        return dx, dw, db


class _Embedding(torch.autograd.Function):
    """F.embedding whose backward is a deterministic scatter into an fp32 [V, H] gradient (csrc/fused_bert.hip
    emb_bwd_chunks / emb_bwd_combine: an id's occurrences summed in token order, in chunks of 64 on separate
    workgroups, the chunks added in order; index_add_ elsewhere), not the sort +
    unique-by-key (rocPRIM partition with decoupled look-back) of PyTorch's embedding backward: that kernel
    faults under hipGraph replay on ROCm (HSA_STATUS_ERROR_MEMORY_APERTURE_VIOLATION in
    rocprim::partition_kernel on the first replay of a captured BERT fwd+bwd, diagnosed in round 1), and
    corrupted the captured training step (non-finite loss after ~10 replays). index_add_'s float atomics made runs
    differ in the last bits (repeated positions / tokens), which the deterministic kernels remove. (A first version
    summed each id on ONE workgroup: the two token-type rows, 2048 occurrences each, cost ~0.5 ms per BERT-base step,
    profiles/bert_steady_r4d.md.)"""

    @staticmethod
    def forward(ctx, ids, weight):
        ctx.save_for_backward(ids)
        ctx.wshape, ctx.wdtype = weight.shape, weight.dtype
        return F.embedding(ids, weight)

    @staticmethod
    def backward(ctx, dy):
        (ids,) = ctx.saved_tensors
        V, H = ctx.wshape
        flat = ids.reshape(-1)
        if dy.is_cuda and flat.numel() <= 32768 and dy.dtype in (torch.float32, torch.bfloat16) \
                and ctx.wdtype in (torch.float32, torch.bfloat16):
            # rows written in the weight's dtype: no fp32 [V, H] image and cast (the word embedding's is 94 MB)
            g = torch.zeros(V, H, device=dy.device, dtype=ctx.wdtype)
            idl = flat.to(torch.int64).contiguous()
            d2 = dy.reshape(-1, H).contiguous()
            part = torch.empty(idl.numel(), H, device=dy.device, dtype=torch.float32)
            heavy = torch.empty(idl.numel(), device=dy.device, dtype=torch.int32)
            check(_fns()["emb_bwd"](int(d2.dtype == torch.bfloat16), ptr(idl), idl.numel(), ptr(d2), H, V, ptr(g),
                                    int(g.dtype == torch.bfloat16), ptr(part), ptr(heavy), stream_handle(dy.device)),
                  "mifx_bert_emb_bwd")
            return None, g
        g = torch.zeros(V, H, device=dy.device, dtype=torch.float32)
        g.index_add_(0, flat, dy.reshape(-1, H).float())
        return None, g.to(ctx.wdtype)


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Embedding lookup with a hipGraph-safe dense backward on the GPU."""
    if ids.is_cuda and not _TORCH_OPS:
        return _Embedding.apply(ids, weight)
    return F.embedding(ids, weight)


def bias_add(y: torch.Tensor, bias: torch.Tensor) -> torch.Tensor:
    if y.is_cuda and not _TORCH_OPS:
        return _BiasAdd.apply(y, bias)
    return y + bias.to(y.dtype)


def linear(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None) -> torch.Tensor:
    """F.linear with a deterministic HIP bias-gradient reduction on the GPU."""
    if x.is_cuda and bias is not None and not _TORCH_OPS:
        return _Linear.apply(x, weight, bias)
    return F.linear(x, weight, bias)


# diagnostic switch: MIFX_BERT_TORCH_OPS=1 runs the PyTorch reference ops on the GPU too (bisection only)
_TORCH_OPS = os.environ.get("MIFX_BERT_TORCH_OPS") == "1"


def bias_dropout_add_layernorm(a: torch.Tensor, bias, r: torch.Tensor, weight, ln_bias, eps: float = 1e-12,
                               p: float = 0.0, rng: torch.Tensor | None = None, site: int = 0,
                               slot=None, eoff: int = 0) -> torch.Tensor:
    """LayerNorm(dropout_p(a + bias) + r) * weight + ln_bias (bias optional; p > 0 needs rng = device int64
    [seed, counter]). The mask depends only on (seed, counter, site, element index): every tensor-parallel rank
    with the same seed drops the same elements of a replicated activation, and a captured hipGraph draws a new
    mask per replay once the counter is advanced in-graph. slot (mifx.ops.gemm.GradSlot, GPU path only): the
    residual's gradient is handed to the projection that also reads r instead of being returned to autograd."""
    if p > 0 and rng is None:
        raise ValueError("dropout p > 0 needs an rng state tensor [seed, counter]")
    if a.is_cuda and not _TORCH_OPS:
        return _BiasDropAddLN.apply(a, bias, r, weight, ln_bias, eps, p, rng, site, slot, eoff)
    if slot is not None:
        raise ValueError("a residual-gradient slot needs the fused GPU path")
    x = a if bias is None else a + bias.to(a.dtype)
    if p > 0:  # (eoff: this tensor is the slice [eoff, eoff + numel) of a larger activation's mask)
        keep = _mask(eoff + x.numel(), rng, site, p, x.device)[eoff:].view(x.shape)
        x = torch.where(keep, x * _drop_scale(p), torch.zeros((), dtype=x.dtype, device=x.device))
    return F.layer_norm(x + r, (a.shape[-1],), weight, ln_bias, eps)


def add_layernorm(a: torch.Tensor, r: torch.Tensor, weight, bias, eps: float = 1e-12) -> torch.Tensor:
    """LayerNorm(a + r) * weight + bias."""
    return bias_dropout_add_layernorm(a, None, r, weight, bias, eps)


def dropout(x: torch.Tensor, p: float, rng: torch.Tensor, site: int) -> torch.Tensor:
    """Counter-based dropout with the same mask function as bias_dropout_add_layernorm."""
    if not p > 0:
        return x
    if x.is_cuda and not _TORCH_OPS:
        return _Dropout.apply(x, p, rng, site)
    keep = keep_mask(x.numel(), rng, site, p).to(x.device).view(x.shape)
    return torch.where(keep, x * _drop_scale(p), torch.zeros((), dtype=x.dtype, device=x.device))


def bias_gelu(x: torch.Tensor, bias) -> torch.Tensor:
    """GELU(erf)(x + bias)."""
    if x.is_cuda and not _TORCH_OPS:
        return _BiasGelu.apply(x, bias)
    return F.gelu(x + bias)


# ---- fused attention (csrc/attention.hip) ----------------------------------------------------------------------
@functools.lru_cache(maxsize=None)
def _attn_fns():
    lib = _lib.load("attention")
    return {
        "fwd": sig(lib, "mifx_attn_fwd", [VP, VP, I32, I32, I32, I32, I32, F32, F32, VP, I32, VP, VP, VP]),
        "bwd": sig(lib, "mifx_attn_bwd", [VP, VP, VP, VP, VP, I32, I32, I32, I32, I32, F32, F32, VP, I32, VP, VP,
                                          VP]),
    }


ATTN_SEQ = (64, 128)  # sequence lengths of the one-workgroup-per-head kernels (head dim 64)
ATTN_MAX_SEQ = 512  # longer S (multiple of 64, up to this) run the chunked kernels of the same file


def attn_native_seq(S: int) -> bool:
    return S in ATTN_SEQ or (128 < S <= ATTN_MAX_SEQ and S % 64 == 0)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, kbias, scale, p, rng, site, h0, htot):
        B, S, _, H, Dh = qkv.shape
        qkv = qkv.contiguous()
        out = torch.empty(B, S, H, Dh, device=qkv.device, dtype=torch.bfloat16)
        lse = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32)
        kb = None if kbias is None else kbias.float().contiguous()
        check(_attn_fns()["fwd"](ptr(qkv), ptr(kb), B, S, H, int(h0), int(htot), float(scale), float(p),
                                 ptr(rng if p > 0 else None), int(site), ptr(out), ptr(lse), stream_handle(qkv.device)),
              "mifx_attn_fwd")
        ctx.save_for_backward(qkv, kb, out, lse)
        ctx.args = (float(scale), float(p), _snap(rng, p), int(site), int(h0), int(htot))
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, kb, out, lse = ctx.saved_tensors
        scale, p, rng, site, h0, htot = ctx.args
        B, S, _, H, Dh = qkv.shape
        dout = dout.to(torch.bfloat16).contiguous()
        dqkv = torch.empty_like(qkv)
        dsum = torch.empty(B, H, S, device=qkv.device, dtype=torch.float32) if S > 128 else None
        check(_attn_fns()["bwd"](ptr(qkv), ptr(kb), ptr(out), ptr(dout), ptr(lse), B, S, H, h0, htot, scale, p,
                                 ptr(rng if p > 0 else None), site, ptr(dqkv), ptr(dsum), stream_handle(qkv.device)),
              "mifx_attn_bwd")
        return dqkv, None, None, None, None, None, None, None


def attention_reference(qkv: torch.Tensor, kbias, scale: float, p: float = 0.0, rng=None, site: int = 0, h0: int = 0,
                        htot: int | None = None) -> torch.Tensor:
    """PyTorch reference of the fused attention: qkv [B, S, 3, H, Dh] -> [B, S, H, Dh]; kbias [B, S] additive
    key bias; dropout mask element (b, global head, i, j) = keep_mask at flat index ((b Htot + h0 + h) S + i) S + j
    (the kernel's indexing, so any head split over TP ranks draws the same mask)."""
    B, S, _, H, Dh = qkv.shape
    htot = H if htot is None else htot
    q, k, v = (t.float() for t in qkv.unbind(2))
    s = torch.einsum("bihd,bjhd->bhij", q, k) * scale
    if kbias is not None:
        s = s + kbias.float()[:, None, None, :]
    pr = torch.softmax(s, -1)
    if p > 0:
        keep = _mask(B * htot * S * S, rng, site, p, pr.device).view(B, htot, S, S)[:, h0:h0 + H]
        pr = torch.where(keep, pr * _drop_scale(p), torch.zeros((), dtype=pr.dtype, device=pr.device))
    return torch.einsum("bhij,bjhd->bihd", pr, v.float()).to(qkv.dtype)


def attention(qkv: torch.Tensor, kbias, scale: float, p: float = 0.0, rng=None, site: int = 0, h0: int = 0,
              htot: int | None = None) -> torch.Tensor:
    """Multi-head self-attention over the fused projection output qkv [B, S, 3, H, Dh] -> [B, S, H, Dh].
    GPU (bf16, Dh 64, S 64 / 128, or a multiple of 64 up to 512): csrc/attention.hip fwd/bwd; elsewhere the
    reference composition (same mask)."""
    if p > 0 and rng is None:
        raise ValueError("attention dropout p > 0 needs an rng state tensor [seed, counter]")
    htot = qkv.shape[3] if htot is None else htot
    from . import native_stats

    if (qkv.is_cuda and not _TORCH_OPS and attn_native_seq(qkv.shape[1]) and qkv.shape[4] == 64
            and qkv.dtype == torch.bfloat16):
        native_stats.count("attention", True)
        return _Attention.apply(qkv, kbias, scale, p, rng, site, h0, htot)
    if qkv.is_cuda:
        native_stats.count("attention", False)
    if qkv.is_cuda and not p > 0:  # other shapes without dropout: the library flash kernel, no S x S tensor
        q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
        am = None if kbias is None else kbias[:, None, None, :].to(q.dtype)
        return F.scaled_dot_product_attention(q, k, v, attn_mask=am, scale=scale).transpose(1, 2)
    # with dropout: the reference composition, its counter-based mask drawn on the device (graph-capturable)
    return attention_reference(qkv, kbias, scale, p, rng, site, h0, htot)
