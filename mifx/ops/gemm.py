"""Hand-written gfx950 MFMA GEMM (csrc/gemm.hip): Y = X W^T [+ bias] [-> GELU] for nn.Linear-shaped products.

`linear(x, w, bias)` and `linear_bias_gelu(x, w, bias)` are autograd functions whose FORWARD runs the HIP kernel
(with the bias / bias + GELU epilogue fused) where preferred, and whose backward takes dX = dY W from the library and
dW = dY^T X from the hand-written TN kernel (csrc/gemm_tn.hip) where that is preferred (plus, for GELU, the existing
fused bias-GELU backward kernel: the forward saves exactly what mifx.ops.fused_bert._BiasGelu saves). Shapes the kernel does not tile (M % BM, N % BN, K % 64) take F.linear.

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
from . import native_stats
from ._lib import I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("gemm")
    return {
        "configs": sig(lib, "mifx_gemm_configs", [VP, I32]),
        "nt": sig(lib, "mifx_gemm_nt", [I32, I32, I32, VP, VP, VP, VP, VP, I32, I32, I32, VP]),
        "tr": sig(lib, "mifx_transpose_bf16", [VP, VP, I32, I32, VP]),
        "gelu_bwd": sig(lib, "mifx_gemm_nt_gelu_bwd", [I32, I32, VP, VP, VP, VP, VP, VP, I32, I32, I32, VP]),
        "tr_batch": sig(lib, "mifx_transpose_bf16_batch", [VP, I32, I32, VP]),
    }


class TransposeCache:
    """Transposed copies of a model's projection weights, refreshed in ONE launch per step (csrc/gemm.hip
    transpose_batch), for the dX GEMMs that run as NT products against W^T. Refreshing per step in one kernel replaces
    a transpose launch per weight in the backward (47 per BERT-base step, ~200 us: profiles/archive/bert_steady_r4b.md). The
    owner (BertTrainer) calls refresh() right before every backward -- from the weights as they are then, so a weight
    change of any kind between steps (update, load_state_dict) is seen -- and runs the backward inside
    `use_transposes(cache)`."""

    def __init__(self, weights):
        self.items = {}
        rows, tile0 = [], 0
        for w in weights:
            R, C = w.shape
            if not (w.is_cuda and w.dtype == torch.bfloat16 and w.is_contiguous() and R % 64 == 0 and C % 64 == 0):
                continue
            wt = torch.empty(C, R, device=w.device, dtype=torch.bfloat16)
            self.items[w.data_ptr()] = (tuple(w.shape), wt, w)
            rows.append([w.data_ptr(), wt.data_ptr(), R + (C << 32), tile0])
            tile0 += (R // 64) * (C // 64)
        self.n, self.tiles = len(rows), tile0
        self.table = torch.tensor(rows, dtype=torch.int64).to(next(iter(self.items.values()))[1].device) \
            if rows else None

    def refresh(self) -> None:
        if self.n:
            check(_fns()["tr_batch"](ptr(self.table), self.n, self.tiles, stream_handle(self.table.device)),
                  "mifx_transpose_bf16_batch")

    def get(self, w: torch.Tensor) -> torch.Tensor | None:
        e = self.items.get(w.data_ptr())
        return e[1] if e is not None and e[0] == tuple(w.shape) else None


class use_transposes:
    """Context: _dx / the fused FFN backward take W^T from `cache` (None: no-op) while it is active -- the owner's
    backward runs inside it, so a cache is never consulted for another model's weights."""

    def __init__(self, cache: TransposeCache | None):
        self.cache = cache

    def __enter__(self):
        if self.cache is not None:
            _TCACHES.append(self.cache)
        return self

    def __exit__(self, *exc):
        if self.cache is not None:
            _TCACHES.remove(self.cache)
        return False


_TCACHES: list[TransposeCache] = []


def transposed(w: torch.Tensor) -> torch.Tensor:
    """W^T for an NT dX GEMM: the active TransposeCache's copy when it holds w, else a fresh transpose."""
    for c in _TCACHES:
        wt = c.get(w)
        if wt is not None:
            return wt
    return transpose(w)


def transpose(w: torch.Tensor) -> torch.Tensor:
    """w [R, C] bf16 -> w^T [C, R] contiguous (csrc/gemm.hip transpose_bf16 where R, C % 64 == 0)."""
    R, C = w.shape
    if not (w.is_cuda and w.dtype == torch.bfloat16 and R % 64 == 0 and C % 64 == 0):
        return w.t().contiguous()
    w = w.contiguous()
    out = torch.empty(C, R, device=w.device, dtype=torch.bfloat16)
    check(_fns()["tr"](ptr(w), ptr(out), R, C, stream_handle(w.device)), "mifx_transpose_bf16")
    return out


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
# profiles/archive/gemm_hip_r3b.jsonl; BERT-base, 4096 tokens): attention-out 4096x768x768 10.7 us vs 20.5 us. Measured
# slower there and left on hipBLASLt: QKV 22.9 vs 21.6 us, FFN-in 25.3 vs 23.3 us (with the bias + GELU epilogue
# 37.5 vs 34.9 us for GEMM + separate bias_gelu: the epilogue's second 25 MB output (the pre-bias product the
# backward needs) is written after the last K-tile by every workgroup at once, un-overlapped, and a branch-free erf
# did not change that: profiles/archive/gemm_hip_r3c_fasterf.jsonl), FFN-out 28.9 vs 25.1 us. MIFX_HIP_GEMM=all routes every
# eligible shape to the kernel (heuristic configuration) for A/B runs.
TUNED: dict[tuple[int, int, int], int] = {(4096, 768, 768): 13}
# forward products routed to the 8-wave pipelined kernel (csrc/gemm8.hip) instead: (M, N, K) -> gemm8 configuration.
# MIFX_G8_FWD=1 (A/B) routes BERT-base's QKV / FFN-in / FFN-out shapes at 4096 tokens to the 256 x 256 tiles
# (profiles/bert_fwd_routes_r5.jsonl: QKV 24.3 us standalone vs hipBLASLt 21.1, but 33.6 us per call inside the step
# on the bundled TunableOp solution, profiles/bert_steady_r5.md)
G8_FWD: dict[tuple[int, int, int], int] = {}
_g8f = os.environ.get("MIFX_G8_FWD", "")
if _g8f == "1":
    G8_FWD.update({(4096, 2304, 768): 0, (4096, 3072, 768): 0, (4096, 768, 3072): 3})
elif _g8f:  # "M:N:K=cfg+..." (A/B sweeps)
    for _item in _g8f.split("+"):
        _shape, _cfg = _item.split("=")
        G8_FWD[tuple(int(v) for v in _shape.split(":"))] = int(_cfg)


def _g8_fwd(M: int, N: int, K: int) -> int | None:
    return G8_FWD.get((M, N, K))


def fwd_nt(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, epi: int = 0):
    """The forward product on the routed hand-written kernel: gemm8 where G8_FWD names the shape, else csrc/gemm.hip
    (same (Y, Z) contract: epi 0 / 1 bias / 2 bias + GELU with Z)."""
    cfg = _g8_fwd(x2.shape[0], w.shape[0], x2.shape[1])
    if cfg is not None:
        return gemm8_nt(x2, w, bias, epi, cfg=cfg)
    return gemm_nt(x2, w, bias, epi)


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
    return x.shape[-1] == K and (pick_config(M, N, K) is not None or (M, N, K) in G8_FWD)


def preferred(x: torch.Tensor, w: torch.Tensor) -> bool:
    """Eligible AND measured faster than the library for this shape (TUNED), or MIFX_HIP_GEMM=all."""
    if not eligible(x, w):
        return False
    if os.environ.get("MIFX_HIP_GEMM") == "all":
        return True
    key = (x.numel() // x.shape[-1], *w.shape)
    return key in TUNED or key in G8_FWD


def gemm_nt(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, epi: int = 0,
            cfg: int | None = None) -> tuple[torch.Tensor, torch.Tensor | None]:
    """x2 [M, K] bf16, w [N, K] bf16 -> (Y [M, N] bf16, Z or None). epi 0: X W^T; 1: + bias; 2: GELU(X W^T + bias)
    with Z = bf16(X W^T) (pre-bias); 3: X W^T + bias where `bias` is a bf16 [M, N] matrix (added before the one
    rounding)."""
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
    if epi == 3:
        b = bias.reshape(M, N).to(torch.bfloat16).contiguous()
    elif epi:
        b = bias if bias.dtype in (torch.float32, torch.bfloat16) else bias.float()
        b = b.contiguous()
    check(_fns()["nt"](int(cfg), int(epi), int(b is not None and b.dtype == torch.float32), ptr(x2), ptr(w), ptr(b),
                       ptr(y), ptr(z), M, N, K, stream_handle(x2.device)), "mifx_gemm_nt")
    return y, z


# Asynchronous weight gradients (opt-in, `async_weight_grads()` context): dW is off the backward's critical path
# (nothing in the backward reads it), so its GEMM is issued on a side stream that forks from the backward stream
# and runs beside the following dX / attention / elementwise kernels; `join_weight_grads()` (before the optimizer)
# joins it. The operands are kept referenced until the join, so the allocator cannot hand their memory to the main
# stream while the side stream still reads them; the dW tensors come from the side stream's pool. Measured SLOWER in
# the BERT-base step (6.75 vs 6.41 ms, identical loss: profiles/archive/bert_async_dw_ab_r3.txt) -- the side-stream GEMMs take
# CUs from the dX GEMMs and attention kernels rather than filling idle ones -- so BertTrainer keeps it off
# (MIFX_BERT_ASYNC_DW=1 turns it on).
_ASYNC = {"on": False, "side": {}, "pending": {}}


class async_weight_grads:
    def __enter__(self):
        self.prev = _ASYNC["on"]
        _ASYNC["on"] = True
        return self

    def __exit__(self, *exc):
        _ASYNC["on"] = self.prev
        return False


def join_weight_grads(device) -> None:
    """The current stream waits for every asynchronous weight gradient issued on `device`."""
    dev = torch.device(device)
    if _ASYNC["pending"].pop(dev, None) is not None:
        torch.cuda.current_stream(dev).wait_stream(_ASYNC["side"][dev])


def _dw_tensor(dy2: torch.Tensor, x2: torch.Tensor) -> torch.Tensor:
    if tn_preferred(dy2.shape[1], x2.shape[1], dy2.shape[0]) and tn_eligible(dy2, x2):
        native_stats.count("gemm_dW", True)
        return gemm_tn(dy2, x2)
    native_stats.count("gemm_dW", False)
    return dy2.t() @ x2


# Deferred weight gradients (`deferred_weight_grads()` context + `flush_weight_grads()`): nothing in a backward reads
# a weight gradient, so each dW = dY^T X is only RECORDED during the backward (its operands kept alive, an empty
# gradient tensor returned to autograd) and all of them run at the end as ONE grouped launch of the pipelined TN
# kernel (csrc/gemm8.hip gemm8_tn_grouped): full 256 x 256 tiles over the whole token reduction, no split-K partials
# and no second summing kernel, instead of one small launch per weight (BERT-base: 48 per step). The flush writes each
# result into the weight's .grad -- whatever tensor autograd ended up storing there -- so the gradients must be reset
# (None or zero) before the backward and each weight may receive ONE recorded product per flush.
_DEFER: dict = {"on": False, "pending": [], "pending_f32": [], "view_of": None}
# token rows per split-K item of the fp32 (convolution) weight gradients; MIFX_WGRAD_CHUNK overrides (A/B)
_WGRAD_CHUNK = int(os.environ.get("MIFX_WGRAD_CHUNK", "4096"))


class deferred_weight_grads:
    """view_of: optional callable weight -> a FRESH tensor view of the memory that should hold its gradient (the
    data-parallel bucket view, mifx.parallel.ddp.DataParallel.grad_view), or None. A weight whose .grad is None then
    gets that view as its placeholder: autograd adopts it as .grad (no copy, no zero-fill + add) and the flush writes the
    product straight into the bucket."""

    def __init__(self, view_of=None):
        self.view_of = view_of

    def __enter__(self):
        self.prev = (_DEFER["on"], _DEFER.get("view_of"))
        _DEFER["on"] = True
        _DEFER["view_of"] = self.view_of
        return self

    def __exit__(self, *exc):
        _DEFER["on"], _DEFER["view_of"] = self.prev
        return False


def _placeholder(w: torch.Tensor) -> tuple[torch.Tensor, bool]:
    """(placeholder gradient for autograd, overwrite). w.grad None: autograd stores the returned tensor as .grad
    untouched, so it may be uninitialised -- the bucket view when a provider gives one -- and the flush OVERWRITES it;
    otherwise autograd adds the placeholder into the existing gradient (micro-batch accumulation): zeros, and the flush
    ADDS."""
    if w.grad is not None:
        return torch.zeros_like(w), False
    vf = _DEFER.get("view_of")
    v = vf(w) if vf is not None else None
    if v is not None and v.shape == w.shape and v.stride() == w.stride() and v.dtype == w.dtype:
        return v, True
    return torch.empty_like(w), True


def grad_destination(p: torch.Tensor) -> torch.Tensor | None:
    """Inside deferred_weight_grads(view_of=...): the memory p's gradient should be written into (the data-parallel
    bucket view) when autograd will adopt the returned tensor as p.grad (p.grad is None), for backward kernels that
    produce a parameter gradient themselves (BatchNorm's dgamma / dbeta: written straight into the bucket instead of
    into a fresh tensor that autograd then adds or the bucket hook copies in). None otherwise."""
    if not _DEFER["on"] or p.grad is not None:
        return None
    vf = _DEFER.get("view_of")
    v = vf(p) if vf is not None else None
    if v is not None and v.shape == p.shape and v.dtype == torch.float32 and v.is_contiguous():
        return v
    return None


def pending_work(weights) -> int:
    """Approximate workgroup count of the grouped flush of these weights' recorded fp32 products (256 x 256 output
    tiles, 4x as many where a 128-wide dimension forces the small tiles, times the token chunks): how much of the GPU
    one flush of them would fill (mifx.parallel.ddp coalesces bucket flushes until it is worth a launch)."""
    ids = {id(w) for w in weights}
    n = 0
    for rec in _DEFER.get("pending_f32", []):
        if id(rec[2]) not in ids:
            continue
        dy, w = rec[0], rec[2]
        T, M = dy.shape
        N = w.numel() // M
        aux = rec[4] if len(rec) > 4 else None
        ck = rec[5] if len(rec) > 5 else _WGRAD_CHUNK
        taps = getattr(aux, "mifx_taps", 1) if aux is not None and aux.dtype == torch.uint8 else 1
        small = M % 256 or (N // taps) % 256
        n += -(-M // 256) * -(-N // 256) * (4 if small else 1) * -(-T // ck)
    return n


def pending_weights() -> set:
    """ids of the weights with a recorded (not yet flushed) fp32 weight-gradient product."""
    return {id(rec[2]) for rec in _DEFER.get("pending_f32", [])}


def _defer_ok(dy2: torch.Tensor, x2: torch.Tensor, w) -> bool:
    if not (_DEFER["on"] and w is not None and dy2.is_cuda and dy2.dtype == torch.bfloat16
            and x2.dtype == torch.bfloat16 and os.environ.get("MIFX_DEFER_DW", "1") != "0"):
        return False
    T, N = dy2.shape
    K = x2.shape[1]
    return N % 256 == 0 and K % 256 == 0 and T % 64 == 0 and len(_DEFER["pending"]) < 64


def defer_weight_grad_f32(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor, bnx: torch.Tensor | None = None):
    """Inside `deferred_weight_grads()`: record dW = dY^T X for the fp32-ACCUMULATING grouped flush (convolution
    weights: fp32 parameters, token counts of 10^4-10^6 rows split into chunks) and return the ZERO placeholder
    gradient for autograd (shape / dtype of w; whatever .grad ends up holding, the flush adds the product into it).
    bnx: fp32 [2, K] (scale, shift): the product is dY^T relu(X scale + shift). None when not deferring (or the shape
    does not tile)."""
    if not (_DEFER["on"] and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16
            and w.dtype == torch.float32 and os.environ.get("MIFX_DEFER_DW", "1") != "0"):
        return None
    T, N = dy2.shape
    K = x2.shape[1]
    tiles = (N % 128 == 0 and K % 128 == 0) or (_G8_NARROW and ((N % 256 == 0 and K % 64 == 0)
                                                                 or (N % 64 == 0 and K % 256 == 0)))
    if not tiles or T % 64 or N * K != w.numel():  # (the last two: the narrow 256 x 64 / 64 x 256 tiles)
        return None
    native_stats.count("conv1x1_dW", True)
    ph, overwrite = _placeholder(w)
    rec = (dy2.contiguous(), x2.contiguous(), w, ph.data_ptr() if overwrite else None)
    _DEFER["pending_f32"].append(rec if bnx is None else rec + (bnx, _WGRAD_CHUNK))
    return ph


def defer_conv3x3_weight_grad_f32(dy2: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, pad: int):
    """As defer_weight_grad_f32 for a 3x3 convolution: dy2 [Nb OH OW, Cout] bf16, x the NHWC bf16 input [Nb, H, W, C],
    w the fp32 channels_last [Cout, C, 3, 3] weight; the flush gathers x per output pixel and tap. None when not
    deferring."""
    if not (_DEFER["on"] and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and w.dtype == torch.float32 and w.is_contiguous(memory_format=torch.channels_last)
            and os.environ.get("MIFX_DEFER_DW", "1") != "0"):
        return None
    nb, h, w_, c = x.shape
    cout = w.shape[0]
    # 256 x 256 tiles (C, Cout % 256) in 2048-pixel chunks measured 99-106 us vs MIOpen's 121-138 on ResNet-50's
    # shapes; 128-wide tiles (C = 128) lose to it (167 vs 130 us): left to the library
    # (profiles/conv3x3_routes_r5.jsonl)
    if cout % 256 or c % 256 or dy2.shape[0] % 64:
        return None
    geo = conv_geo(nb, h, w_, c, stride, pad, x.device)
    native_stats.count("conv3x3_dW", True)
    ph, overwrite = _placeholder(w)
    _DEFER["pending_f32"].append((dy2.contiguous(), x.contiguous(), w, ph.data_ptr() if overwrite else None, geo,
                                  2048))
    return ph


def defer_strided1x1_weight_grad_f32(dy2: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int):
    """As defer_conv3x3_weight_grad_f32 for a strided 1x1 convolution (ResNet's projection shortcuts): dy2 [Nb OH OW,
    Cout] bf16, x NHWC bf16 [Nb, H, W, C], w fp32 [Cout, C, 1, 1]; the flush gathers x's pixel (stride oh, stride ow)
    per output row (the center-tap geometry). C and Cout % 256 (full tiles); None otherwise / when not deferring."""
    if not (_DEFER["on"] and dy2.is_cuda and dy2.dtype == torch.bfloat16 and x.dtype == torch.bfloat16
            and w.dtype == torch.float32 and w.is_contiguous() and os.environ.get("MIFX_DEFER_DW", "1") != "0"):
        return None
    nb, h, w_, c = x.shape
    cout = w.shape[0]
    if cout % 256 or c % 256 or c & (c - 1) or dy2.shape[0] % 64:
        return None
    geo = conv_geo(nb, h, w_, c, stride, 1, x.device, center1x1=True)
    native_stats.count("conv1x1_dW", True)
    ph, overwrite = _placeholder(w)
    _DEFER["pending_f32"].append((dy2.contiguous(), x.contiguous(), w, ph.data_ptr() if overwrite else None, geo,
                                  _WGRAD_CHUNK))
    return ph


def flush_weight_grads(weights=None) -> int:
    """Run every recorded weight gradient as one grouped launch into the weights' .grad; returns how many.
    weights: only the fp32 products of these weights (one data-parallel bucket: its exchange can start right after),
    the others stay recorded."""
    pf_all = _DEFER.get("pending_f32", [])
    if weights is not None:
        ids = {id(w) for w in weights}
        pf = [r for r in pf_all if id(r[2]) in ids]
        _DEFER["pending_f32"] = [r for r in pf_all if id(r[2]) not in ids]
    else:
        pf, _DEFER["pending_f32"] = pf_all, []
    nf = 0
    if pf:
        probs, acc = [], []
        for rec in pf:
            dy, x, w, ph = rec[:4]
            aux = rec[4] if len(rec) > 4 else None
            geo = aux if aux is not None and aux.dtype == torch.uint8 else None
            ck = rec[5] if len(rec) > 5 else _WGRAD_CHUNK
            g = w.grad
            lay_ok = g is not None and (g.is_contiguous(memory_format=torch.channels_last)
                                        if geo is not None and geo.mifx_taps == 9 else g.is_contiguous())
            if g is None or g.dtype != torch.float32 or not lay_ok or g.shape != w.shape:
                raise RuntimeError("deferred weight gradients: the fp32 weight's .grad is missing or not contiguous")
            if ph is not None and g.data_ptr() != ph:
                raise RuntimeError("deferred weight gradients: autograd did not keep the uninitialised placeholder "
                                   "as .grad (was the gradient accumulated?)")
            if geo is not None:  # [Cout][3][3][C] storage of the channels_last gradient ([Cout][C]: strided 1x1)
                flat = g.permute(0, 2, 3, 1).reshape(g.shape[0], -1) if geo.mifx_taps == 9 else g.view(g.shape[0], -1)
                probs.append((dy, x, flat, geo, ck))
            elif aux is not None:  # BatchNorm-operand problem
                probs.append((dy, x, g.view(dy.shape[1], x.shape[1]), aux, ck))
            else:
                probs.append((dy, x, g.view(dy.shape[1], x.shape[1])))
            acc.append(ph is None)
        gemm8_tn_grouped(probs, accumulate=acc)
        nf = len(pf)
    if weights is not None:
        return nf
    pend, _DEFER["pending"] = _DEFER["pending"], []
    if not pend:
        return nf
    seen = set()
    for _, _, w in pend:
        if id(w) in seen:
            raise RuntimeError("deferred weight gradients: a weight received two products in one flush")
        seen.add(id(w))
        g = w.grad
        if g is None or g.dtype != torch.bfloat16 or not g.is_contiguous() or g.shape != w.shape:
            raise RuntimeError("deferred weight gradients: the weight's .grad is not the bf16 tensor the backward "
                               "returned (was it accumulated or replaced?)")
    gemm8_tn_grouped([(dy, x, w.grad) for dy, x, w in pend])
    return len(pend) + nf


def _dw(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor | None = None) -> torch.Tensor:
    """Weight gradient dY^T X: recorded for the grouped flush inside `deferred_weight_grads()` (w: the weight whose
    .grad receives it); else the hand-written TN kernel where it measured faster (TN_TUNED), else hipBLASLt; on a
    side stream inside `async_weight_grads()`."""
    if _defer_ok(dy2, x2, w):
        native_stats.count("gemm_dW", True)
        _DEFER["pending"].append((dy2.contiguous(), x2.contiguous(), w))
        return torch.empty(dy2.shape[1], x2.shape[1], device=dy2.device, dtype=torch.bfloat16)
    if not (_ASYNC["on"] and dy2.is_cuda):
        return _dw_tensor(dy2, x2)
    dev = dy2.device
    side = _ASYNC["side"].get(dev)
    if side is None:
        side = _ASYNC["side"][dev] = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        dw = _dw_tensor(dy2, x2)
    _ASYNC["pending"].setdefault(dev, []).append((dy2, x2))
    return dw


def tn_preferred(n_out: int, k_in: int, tokens: int) -> bool:
    return (n_out, k_in, tokens) in TN_TUNED and os.environ.get("MIFX_HIP_GEMM_TN", "1") != "0"


class GradSlot:
    """Hand-off of a residual branch's input gradient into the input-gradient GEMM of the other consumer of the
    same activation. In a BERT layer h feeds both a projection and the residual of the next add+LayerNorm; autograd
    would sum the two gradients with one extra elementwise kernel per activation (2 per layer). Instead the
    add+LayerNorm backward (which always runs first: the projection's output gradient flows through it) parks its
    residual gradient here and returns none, and the projection's backward folds it in as the GEMM's C operand
    (dX = dY W + dR, one addmm). Single tensor-parallel rank only (with TP the dX GEMM output is a partial sum)."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None


# ---------------------------------------------------------------- input-gradient GEMM (csrc/gemm_nn.hip)
@functools.lru_cache(maxsize=None)
def _nn_fns():
    lib = _lib.load("gemm_nn")
    return {"configs": sig(lib, "mifx_gemm_nn_configs", [VP, I32]),
            "nn": sig(lib, "mifx_gemm_nn", [I32, VP, VP, VP, VP, I32, I32, I32, VP])}


@functools.lru_cache(maxsize=None)
def nn_configs() -> tuple[tuple[int, int, int], ...]:
    """(BM, BN, ring depth) of every compiled NN configuration, by index."""
    buf = (ctypes.c_int * 96)()
    n = _nn_fns()["configs"](buf, 96)
    return tuple((buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(n))


# (M, N, K) of dX = dY[M, K] W[K, N] -> configuration, where the NN kernel measured faster than hipBLASLt
# (tools/bench_gemm_hip.py --dx); other shapes stay on the library
NN_TUNED: dict[tuple[int, int, int], int] = {}


def nn_pick(M: int, N: int, K: int, cus: int = 256) -> int | None:
    if (M, N, K) in NN_TUNED:
        return NN_TUNED[(M, N, K)]
    best, best_score = None, None
    for i, (bm, bn, _) in enumerate(nn_configs()):
        if M % bm or N % bn or K % 64:
            continue
        tiles = (M // bm) * (N // bn)
        fill = tiles / (-(-tiles // cus) * cus)
        score = (fill * (bm * bn) ** 0.25, bm * bn)
        if best_score is None or score > best_score:
            best, best_score = i, score
    return best


def gemm_nn(a: torch.Tensor, b: torch.Tensor, r: torch.Tensor | None = None, cfg: int | None = None) -> torch.Tensor:
    """a [M, K] bf16, b [K, N] bf16 (row-major) -> a @ b (+ r [M, N]) bf16 on csrc/gemm_nn.hip (fp32 accumulation,
    r added before the single rounding: torch.addmm(r, a, b)'s contract)."""
    M, K = a.shape
    N = b.shape[1]
    if cfg is None:
        cfg = nn_pick(M, N, K)
    if cfg is None:
        raise ValueError(f"no NN tile configuration for {M}x{N}x{K}")
    a, b = a.contiguous(), b.contiguous()
    if r is not None:
        r = r.reshape(M, N).to(torch.bfloat16).contiguous()
    c = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    check(_nn_fns()["nn"](int(cfg), ptr(a), ptr(b), ptr(r), ptr(c), M, N, K, stream_handle(a.device)), "mifx_gemm_nn")
    return c


def nn_preferred(M: int, N: int, K: int) -> bool:
    if os.environ.get("MIFX_HIP_GEMM_NN", "1") == "0":
        return False
    return (M, N, K) in NN_TUNED or (os.environ.get("MIFX_HIP_GEMM") == "all" and nn_pick(M, N, K) is not None)


# dX = dY[M, K] W[K, N] as an NT product dY . (W^T)^T against a transposed weight copy (transpose_bf16, 1-3 us per
# BERT weight) with the residual gradient folded into the epilogue: measured faster than hipBLASLt's NN kernels and
# much faster than its addmm (the GradSlot fold) on BERT-base's shapes at 4096 tokens
# (profiles/gemm_dx_r4.jsonl): QKV 23.5 vs 30.3 (addmm 35.2) us, attention-out 10.4 vs 19.4, FFN-in 29.7 vs 39.2
# (addmm 70.2). FFN-out (N = 3072) ties and stays on the library. (M, N, K) -> NT configuration.
DX_NT_TUNED: dict[tuple[int, int, int], int] = {(4096, 768, 2304): 13, (4096, 768, 768): 12, (4096, 768, 3072): 13}
# input-gradient products routed to the 8-wave kernel instead (A/B: MIFX_G8_DX="M:N:K=cfg+...", none by default)
G8_DX: dict[tuple[int, int, int], int] = {}
for _item in filter(None, os.environ.get("MIFX_G8_DX", "").split("+")):
    _shape, _cfg = _item.split("=")
    G8_DX[tuple(int(v) for v in _shape.split(":"))] = int(_cfg)


def _dx(dy2: torch.Tensor, w: torch.Tensor, slot: GradSlot | None) -> torch.Tensor:
    """dX = dY W (+ the residual gradient parked in `slot` as the C operand): the hand-written NT kernel against a
    transposed weight copy where it measured faster (DX_NT_TUNED), the NN kernel where tuned (NN_TUNED), else
    hipBLASLt."""
    g = None
    if slot is not None:
        g, slot.g = slot.g, None
        if g is None:
            raise RuntimeError("GradSlot empty: the residual gradient did not arrive before the projection's backward")
    M, K = dy2.shape
    N = w.shape[1]
    ok = dy2.is_cuda and dy2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
    if ok and (M, N, K) in G8_DX:
        native_stats.count("gemm_dX", True)
        y, _ = gemm8_nt(dy2, transposed(w), g, 3 if g is not None else 0, cfg=G8_DX[(M, N, K)])
        return y
    if ok and (M, N, K) in DX_NT_TUNED and os.environ.get("MIFX_HIP_GEMM_DX", "1") != "0":
        native_stats.count("gemm_dX", True)
        y, _ = gemm_nt(dy2, transposed(w), g, 3 if g is not None else 0, cfg=DX_NT_TUNED[(M, N, K)])
        return y
    native = ok and nn_preferred(M, N, K)
    native_stats.count("gemm_dX", native)
    if native:
        return gemm_nn(dy2, w, g)
    if g is None:
        return dy2 @ w
    return torch.addmm(g.reshape(-1, w.shape[1]).to(dy2.dtype), dy2, w)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, hip_fwd=True, slot=None, tp=None, tp_in=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        ctx.tp_in = tp_in
        if tp is not None:  # row-parallel: the product all-reduced over the TP group, overlapped chunk by chunk
            from ..parallel.tensor_parallel import gemm_allreduce_overlapped

            y = gemm_allreduce_overlapped(x2, lambda xc: gemm_nt(xc, w)[0] if hip_fwd else F.linear(xc, w),
                                          w.shape[0], tp)
            if bias is not None:
                y = y + bias.to(y.dtype)
        elif hip_fwd:
            y, _ = fwd_nt(x2, w, bias, 1 if bias is not None else 0)
        else:
            y = F.linear(x2, w, bias)
        ctx.save_for_backward(x2, w)
        ctx.slot = slot
        ctx.has_bias = bias is not None
        ctx.bdtype = bias.dtype if bias is not None else None
        return y.view(*shp[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).to(x2.dtype)
        dx = None
        if ctx.needs_input_grad[0]:
            dx = _dx_reduced(dy2, w, ctx.slot, ctx.tp_in).view(*dy.shape[:-1], w.shape[1])
        dw = _dw(dy2.contiguous(), x2, w) if ctx.needs_input_grad[1] else None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            from .fused_bert import col_sum

            db = col_sum(dy2, ctx.bdtype if ctx.bdtype in (torch.float32, torch.bfloat16) else torch.float32)
        return dx, dw, db, None, None, None, None


def _dx_reduced(dy2: torch.Tensor, w: torch.Tensor, slot, tp_in) -> torch.Tensor:
    """_dx, then (column-parallel input, tp_in) its all-reduce over the TP group -- overlapped with the dX GEMM in
    token chunks on the peer-memory path (mifx.parallel.tensor_parallel.gemm_allreduce_overlapped)."""
    if tp_in is None:
        return _dx(dy2, w, slot)
    from ..parallel import tensor_parallel as tpm

    if slot is None and tpm.overlap_ok(tp_in, dy2.shape[0], w.shape[1]) and dy2.dtype == torch.bfloat16:
        return tpm.gemm_allreduce_overlapped(dy2, lambda dc: _dx(dc, w, None), w.shape[1], tp_in)
    return tpm._all_reduce(_dx(dy2, w, slot), tp_in)


class _LinearBiasGelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, slot=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        y, z = fwd_nt(x2, w, bias, 2)
        ctx.slot = slot
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
        dx = _dx(dz, w, ctx.slot).view(*dy.shape[:-1], w.shape[1]) if ctx.needs_input_grad[0] else None
        dw = _dw(dz, x2, w) if ctx.needs_input_grad[1] else None
        return dx, dw, db if bp.dtype == ctx.bdtype else db.to(ctx.bdtype), None


def linear(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, force: bool = False,
           slot: GradSlot | None = None, tp=None, tp_in=None) -> torch.Tensor:
    """F.linear with the forward on the hand-written kernel (bias fused) where it is preferred (or, force=True,
    wherever it tiles the shape), and the weight gradient on the hand-written TN kernel where that is preferred.
    slot: the input gradient also carries the residual gradient parked there (GradSlot). tp: a row-parallel
    projection whose product is returned ALL-REDUCED over the group, the reduction overlapped with the GEMM in token
    chunks (only where mifx.parallel.tensor_parallel.overlap_ok; elsewhere the caller applies reduce_from_tp). tp_in:
    a column-parallel projection of a replicated input (Megatron's copy_to_tp folded in): the input gradient is
    all-reduced over the group, overlapped with its GEMM in token chunks where possible."""
    fwd = eligible(x, w) if force else preferred(x, w)
    if x.is_cuda:
        native_stats.count("gemm_fwd", fwd)
    bwd = (x.is_cuda and x.dtype == torch.bfloat16 and w.requires_grad and torch.is_grad_enabled()
           and tn_preferred(w.shape[0], w.shape[1], x.numel() // x.shape[-1]))
    if tp is not None or (tp_in is not None and tp_in.size > 1):
        return _Linear.apply(x, w, bias, fwd, slot, tp, tp_in if tp_in is not None and tp_in.size > 1 else None)
    if fwd or bwd or slot is not None:
        return _Linear.apply(x, w, bias, fwd, slot)
    return F.linear(x, w, bias)


def linear_bias_gelu(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, force: bool = False,
                     slot: GradSlot | None = None) -> torch.Tensor:
    """GELU(x w^T + bias) with the bias + GELU fused into the GEMM epilogue where preferred (force: wherever it
    tiles)."""
    if eligible(x, w) if force else preferred(x, w):
        native_stats.count("gemm_fwd_bias_gelu", True)
        return _LinearBiasGelu.apply(x, w, bias, slot)
    if x.is_cuda:
        native_stats.count("gemm_fwd_bias_gelu", False)
    from .fused_bert import bias_gelu

    return bias_gelu(linear(x, w, slot=slot), bias)


# ---------------------------------------------------------------- weight-gradient GEMM (csrc/gemm_tn.hip)
@functools.lru_cache(maxsize=None)
def _tn_fns():
    lib = _lib.load("gemm_tn")
    return {
        "configs": sig(lib, "mifx_gemm_tn_configs", [VP, I32]),
        "tn": sig(lib, "mifx_gemm_tn", [I32, VP, VP, VP, VP, I32, I32, I32, I32, VP]),
    }


@functools.lru_cache(maxsize=None)
def tn_configs() -> tuple[tuple[int, int, int], ...]:
    """(BM, BN, OPT bits) of every compiled TN tile configuration, by index."""
    buf = (ctypes.c_int * 96)()
    n = _tn_fns()["configs"](buf, 96)
    return tuple((buf[3 * i], buf[3 * i + 1], buf[3 * i + 2]) for i in range(n))


# measured per-shape choices (M, N, T) -> (cfg, splits); tools/bench_gemm_tn.py, profiles/archive/gemm_tn_r3.jsonl
# BERT-base at 4096 tokens (B = 32, S = 128), us vs hipBLASLt `dy.t() @ x`: QKV 30.7 vs 36.2, attention-out 18.3 vs
# 27.6, FFN-in 38.0 vs 41.8, FFN-out 37.7 vs 42.6 (configs with 2-3 workgroups per CU and a token split; the one-
# workgroup-per-CU deep-ring configurations measured slower: the per-CU operand stream, not DMA latency, bounds a
# 96 x 96 tile at ~30 GB/s per workgroup; profiles/archive/gemm_tn_r3.jsonl)
TN_TUNED: dict[tuple[int, int, int], tuple[int, int]] = {(2304, 768, 4096): (10, 4), (768, 768, 4096): (9, 8),
                                                         (3072, 768, 4096): (9, 2), (768, 3072, 4096): (9, 2)}


def pick_tn(M: int, N: int, T: int, cus: int = 256) -> tuple[int, int] | None:
    """(config index, token splits) for C[M, N] = A[T, M]^T B[T, N]; None if no configuration tiles it. Splits: the
    largest power of two that keeps tiles x splits within one wave of workgroups (T % (64 splits) == 0)."""
    if (M, N, T) in TN_TUNED:
        return TN_TUNED[(M, N, T)]
    best, best_score = None, None
    for i, (bm, bn, opt) in enumerate(tn_configs()):
        if M % bm or N % bn or T % 64 or opt % 16:  # (the heuristic picks among the plain 4-wave forms)
            continue
        tiles = (M // bm) * (N // bn)
        s = 1
        while tiles * s * 2 <= cus and T % (64 * s * 2) == 0 and T // (s * 2) >= 512:
            s *= 2
        wgs = tiles * s
        fill = wgs / (-(-wgs // cus) * cus)
        score = (round(fill, 3), -abs(bm * bn - 96 * 96))  # full waves first, then the 96 x 96 tile
        if best_score is None or score > best_score:
            best, best_score = (i, s), score
    return best


def gemm_tn(a: torch.Tensor, b: torch.Tensor, cfg: int | None = None, splits: int | None = None) -> torch.Tensor:
    """a [T, M] bf16, b [T, N] bf16 (row-major) -> a^T b [M, N] bf16 with fp32 accumulation (the weight gradient
    dY^T X of a linear layer)."""
    T, M = a.shape
    N = b.shape[1]
    if b.shape[0] != T:
        raise ValueError("a and b must have the same number of rows")
    if cfg is None or splits is None:
        pk = pick_tn(M, N, T)
        if pk is None:
            raise ValueError(f"no TN tile configuration for {M}x{N} over {T} rows")
        cfg = pk[0] if cfg is None else cfg
        splits = pk[1] if splits is None else splits
    a, b = a.contiguous(), b.contiguous()
    c = torch.empty(M, N, device=a.device, dtype=torch.bfloat16)
    part = torch.empty(splits, M, N, device=a.device, dtype=torch.float32) if splits > 1 else None
    check(_tn_fns()["tn"](int(cfg), ptr(a), ptr(b), ptr(c), ptr(part), M, N, T, int(splits),
                          stream_handle(a.device)), "mifx_gemm_tn")
    return c


def tn_eligible(a2: torch.Tensor, b2: torch.Tensor) -> bool:
    return (a2.is_cuda and a2.dtype == torch.bfloat16 and b2.dtype == torch.bfloat16 and a2.dim() == 2
            and b2.dim() == 2 and pick_tn(a2.shape[1], b2.shape[1], a2.shape[0]) is not None)


# ---------------------------------------------------------------- ping-pong pipelined NT GEMM (csrc/gemm8.hip)
@functools.lru_cache(maxsize=None)
def _g8_fns():
    lib = _lib.load("gemm8")
    return {"configs": sig(lib, "mifx_gemm8_configs", [VP, I32]),
            "nt": sig(lib, "mifx_gemm8_nt", [I32, I32, I32, VP, VP, VP, VP, VP, VP, I32, I32, I32, VP, VP]),
            "tn": sig(lib, "mifx_gemm8_tn_grouped", [I32, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP, VP]),
            "conv": sig(lib, "mifx_gemm8_conv3x3", [I32, I32, VP, VP, VP, VP, VP, VP, I32, I32, I32, I32, I32, I32,
                                                    I32, VP]),
            "geo_bytes": sig(lib, "mifx_gemm8_geo_bytes", []),
            "geo": sig(lib, "mifx_gemm8_geo", [I32, I32, I32, I32, I32, I32, I32, VP]),
            "conv1x1s": sig(lib, "mifx_gemm8_conv1x1s", [I32, I32, VP, VP, VP, VP, I32, I32, I32, I32, I32, I32, VP]),
            "nt_bnx": sig(lib, "mifx_gemm8_nt_bnx", [I32, I32, VP, VP, VP, VP, VP, I32, I32, I32, VP, VP])}


@functools.lru_cache(maxsize=None)
def gemm8_configs() -> tuple[tuple[int, int], ...]:
    """(BM, BN) of every compiled csrc/gemm8.hip configuration, by index."""
    buf = (ctypes.c_int * 64)()
    n = _g8_fns()["configs"](buf, 64)
    return tuple((buf[2 * i], buf[2 * i + 1]) for i in range(n))


# Relative throughput of each tile shape when it fills the chip (4096^3: 1174 / 875 / 962 / 866 TFLOP/s, adjusted by
# the ResNet 3x3 / 1x1 sweeps in profiles/conv3x3_routes_r5.jsonl) and workgroups per CU (128 x 128: <= 128 VGPRs and
# 64 KB of LDS, two co-resident)
_G8_EFF = {(256, 256): 1.0, (256, 128): 0.745, (128, 256): 0.78, (128, 128): 0.85, (256, 64): 0.5, (128, 64): 0.45}
_G8_OCC = {(128, 128): 2, (256, 64): 2, (128, 64): 2}
# the 64-wide (narrow) tiles: the only configurations for N = 64 (ResNet-50 stage 1); MIFX_G8_NARROW=0 leaves those
# products to the library (A/B)
_G8_NARROW = os.environ.get("MIFX_G8_NARROW", "1") != "0"


# the BatchNorm-operand (AX) build of the 256 x 256 tile spills registers: left out of its picks unless MIFX_BNX_256=1
_BNX_256 = os.environ.get("MIFX_BNX_256", "0") == "1"


# measured winners for ResNet-50's 1x1 products at B = 256 (tools/bench_gemm8.py --shapes resnet,
# profiles/gemm8_resnet_1x1_configs_r5.jsonl): with K <= 512 the 128 x 128 tiles (two workgroups per CU, so one's
# epilogue overlaps the other's loads) beat the 256 x 256 tiles the throughput heuristic prefers -- e.g. 802816 x 256 x 64
# 118.9 vs 136.1 us, 50176 x 1024 x 256 41.4 vs 49.2, 12544 x 512 x 2048 33.7 vs 44.4. MIFX_G8_TUNED=0: heuristic only
_G8_TUNED_ON = os.environ.get("MIFX_G8_TUNED", "1") != "0"
_G8_TUNED: dict[tuple[int, int, int], tuple[int, int]] = {
    (802816, 256, 64): (128, 128), (200704, 128, 512): (128, 128), (200704, 512, 128): (128, 128),
    (50176, 256, 1024): (256, 256), (50176, 1024, 256): (128, 128), (12544, 512, 2048): (128, 128),
    (12544, 2048, 512): (256, 256),
}


def gemm8_pick(M: int, N: int, K: int, cus: int = 256, bnx: bool = False) -> int | None:
    """The csrc/gemm8.hip configuration for an M x N x K product: a measured winner (_G8_TUNED), else the highest
    (fraction of the last wave's slots filled) x (the tile's relative throughput); None if none tiles the shape.
    bnx: for gemm8_nt_bnx."""
    t = _G8_TUNED.get((M, N, K)) if _G8_TUNED_ON else None
    if t is not None and not (bnx and t == (256, 256) and not _BNX_256):
        cfgs = gemm8_configs()
        if t in cfgs:
            return cfgs.index(t)
    best, best_score = None, None
    for i, (bm, bn) in enumerate(gemm8_configs()):
        if M % bm or N % bn or K % 64 or (bn == 64 and not _G8_NARROW):
            continue
        if bnx and (bm, bn) == (256, 256) and not _BNX_256:
            continue
        tiles = (M // bm) * (N // bn)
        slots = cus * _G8_OCC.get((bm, bn), 1)
        waves = -(-tiles // slots)
        score = (tiles / (waves * slots) * _G8_EFF.get((bm, bn), 0.5), bm * bn)
        if best_score is None or score > best_score:
            best, best_score = i, score
    return best


_G8_MAXP = 48  # problems per grouped launch (the table travels in the kernel arguments)


def gemm8_tn_grouped(problems, chunk: int = 4096, tile128: bool | None = None, accumulate=True) -> int:
    """problems: [(a [T, M], b [T, N], c [M, N]), ...] CUDA tensors on one device (a, b bf16) -> for every problem, in
    ONE launch of csrc/gemm8.hip's pipelined TN kernel: c = a^T b when c is bf16; c += a^T b when c is fp32 (c = a^T b
    where `accumulate` -- a bool or one per problem -- is False), the token range cut into `chunk`-row pieces whose
    fp32 partials a second launch sums in order. 256 x 256 tiles where M and N allow (tile128=True forces 128 x 128).
    A 4-tuple (dy [T, Cout], x NHWC [Nb, H, W, C], c fp32 [Cout, 9 C], geo) is a 3x3 convolution's weight gradient
    with the input rows gathered per output pixel and tap (geo = conv_geo(...)); (a, b, c fp32, ax) with ax an fp32
    [2, N] (scale, shift) multiplies a by relu(b scale + shift) instead of b (a BatchNorm + ReLU input whose output was
    never stored, mifx.ops.conv1x1.bn_conv1x1). A 5th element: the problem's token chunk. Returns the work items."""
    n = len(problems)
    if n == 0:
        return 0
    accs = list(accumulate) if isinstance(accumulate, (list, tuple)) else [bool(accumulate)] * n
    if n > _G8_MAXP:
        return sum(gemm8_tn_grouped(problems[i:i + _G8_MAXP], chunk, tile128, accs[i:i + _G8_MAXP])
                   for i in range(0, n, _G8_MAXP))
    Ms, Ns, Ts, chunks, flags, geos, ws_floats = [], [], [], [], [], [], 0
    for pr in problems:
        a, b, c = pr[:3]
        aux = pr[3] if len(pr) > 3 else None
        bnx = aux if aux is not None and aux.dtype == torch.float32 else None  # BatchNorm (scale, shift) of B
        geo = aux if bnx is None else None
        pchunk = pr[4] if len(pr) > 4 else chunk
        taps = getattr(geo, "mifx_taps", 9)
        if geo is not None:
            T, M = a.shape
            N = c.numel() // M
            if not (a.is_contiguous() and b.is_contiguous() and a.dtype == torch.bfloat16
                    and b.dtype == torch.bfloat16 and c.dtype == torch.float32 and N * M == c.numel()
                    and N % taps == 0 and b.shape[-1] == N // taps):
                raise ValueError("gemm8_tn_grouped: a conv problem needs bf16 dy [T, Cout], NHWC bf16 x [.., C] and "
                                 "fp32 c [Cout, taps C]")
        else:
            if not (a.is_contiguous() and b.is_contiguous() and c.is_contiguous()) or a.shape[0] != b.shape[0] or \
                    c.numel() != a.shape[1] * b.shape[1] or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16 \
                    or c.dtype not in (torch.bfloat16, torch.float32):
                raise ValueError("gemm8_tn_grouped: need contiguous bf16 a [T, M], b [T, N] and c [M, N] (bf16 / "
                                 "fp32)")
            T, M = a.shape
            N = b.shape[1]
            if bnx is not None and not (c.dtype == torch.float32 and bnx.is_contiguous() and bnx.numel() == 2 * N):
                raise ValueError("gemm8_tn_grouped: a BatchNorm-operand problem needs fp32 c and fp32 [2, N] scale / "
                                 "shift")
        f32 = c.dtype == torch.float32
        t128 = tile128 if tile128 is not None else (M % 256 or N % 256 or (geo is not None and (N // taps) % 256))
        # a 64-wide dimension (ResNet-50 stage 1): the narrow 256 x 64 / 64 x 256 tiles (fp32 problems)
        cw = N // taps if geo is not None else N
        nar_n = _G8_NARROW and f32 and tile128 is None and cw % 128 and cw % 64 == 0 and M % 256 == 0
        nar_m = _G8_NARROW and f32 and tile128 is None and geo is None and M % 128 and M % 64 == 0 \
            and N % 256 == 0
        if nar_n or nar_m:
            t128 = False
        elif bnx is not None:  # (the kernel builds BatchNorm-operand problems on 128 x 128 or narrow tiles only)
            t128 = True
        ck = pchunk if f32 else T
        Ms.append(M)
        Ns.append(N)
        Ts.append(T)
        chunks.append(ck)
        flags.append((1 if f32 else 0) | (2 if t128 else 0) | (4 if f32 and accs[len(flags)] else 0)
                     | (8 if geo is not None else 0) | (16 if nar_n else 0) | (32 if nar_m else 0)
                     | (64 if bnx is not None else 0))
        geos.append(aux.data_ptr() if aux is not None else None)
        if f32:
            ws_floats += -(-T // ck) * M * N
    dev = problems[0][0].device
    ws = torch.empty(ws_floats, device=dev, dtype=torch.float32) if ws_floats else None
    arr = lambda xs, t=ctypes.c_int: (t * n)(*xs)  # noqa: E731
    rc = _g8_fns()["tn"](n, arr([pr[0].data_ptr() for pr in problems], VP),
                         arr([pr[1].data_ptr() for pr in problems], VP),
                         arr([pr[2].data_ptr() for pr in problems], VP), arr(Ms), arr(Ns), arr(Ts), arr(chunks),
                         arr(flags), ptr(ws), arr(geos, VP), stream_handle(dev))
    if rc <= 0:
        raise RuntimeError(f"mifx_gemm8_tn_grouped failed ({rc})")
    return rc


_GEO: dict = {}


def conv_geo(nb: int, h: int, w: int, c: int, stride: int, pad: int, device, center1x1: bool = False) -> torch.Tensor:
    """The device-resident geometry record of a 3x3 convolution -- or, center1x1, of a strided 1x1 one (the center
    tap of a pad-1 3x3: weight gradient [Cout, C]) -- for the grouped weight-gradient launch (created once per shape,
    before any graph capture reads it; `.mifx_taps` = taps per weight row)."""
    key = (nb, h, w, c, stride, pad, bool(center1x1), str(device))
    g = _GEO.get(key)
    if g is None:
        nbytes = _g8_fns()["geo_bytes"]()
        host = (ctypes.c_ubyte * nbytes)()
        if _g8_fns()["geo"](nb, h, w, c, stride, pad, int(bool(center1x1)), host) != 0:
            raise ValueError(f"no convolution geometry for {key}")
        g = torch.tensor(list(bytes(host)), dtype=torch.uint8).to(device)
        g.mifx_taps = 1 if center1x1 else 9
        _GEO[key] = g
    return g


def gemm8_conv1x1_strided(x: torch.Tensor, w: torch.Tensor, stride: int = 2, epi: int = 0, cfg: int | None = None,
                          out: torch.Tensor | None = None):
    """Strided 1x1 convolution of NHWC bf16 x [Nb, H, W, C] (C a power of two >= 64) with w [Cout, C] bf16 on
    csrc/gemm8.hip (the center tap of the implicit 3x3 GEMM) -> (y [Nb OH OW, Cout] bf16, part); epi 5: part = per-tile
    BatchNorm statistics of y."""
    nb, h, w_, c = x.shape
    cout = w.shape[0]
    oh, ow = (h - 1) // stride + 1, (w_ - 1) // stride + 1
    M = nb * oh * ow
    if cfg is None:
        cfg = gemm8_pick(M, cout, c)
    if cfg is None:
        raise ValueError(f"no gemm8 tile configuration for the {M}x{cout}x{c} strided convolution")
    if not (x.is_contiguous() and w.is_contiguous() and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and tuple(w.shape) == (cout, c)):
        raise ValueError("gemm8_conv1x1_strided: contiguous bf16 NHWC input and [Cout, C] weight")
    bm = gemm8_configs()[cfg][0]
    y = out if out is not None else torch.empty(M, cout, device=x.device, dtype=torch.bfloat16)
    part = torch.empty(2, M // bm, cout, device=x.device, dtype=torch.float32) if epi == 5 else None
    check(_g8_fns()["conv1x1s"](int(cfg), int(epi), ptr(x), ptr(w), ptr(y), ptr(part), nb, h, w_, c, cout, stride,
                                stream_handle(x.device)), "mifx_gemm8_conv1x1s")
    return y, part


def gemm8_conv3x3(x: torch.Tensor, w9: torch.Tensor, stride: int = 1, pad: int = 1, epi: int = 0,
                  cfg: int | None = None, bias: torch.Tensor | None = None, z: torch.Tensor | None = None,
                  out: torch.Tensor | None = None):
    """3x3 convolution of NHWC bf16 x [Nb, H, W, C] (C a power of two >= 64) with w9 [Cout, 9 C] bf16 (a
    channels_last [Cout, C, 3, 3] weight's storage) as an implicit GEMM on csrc/gemm8.hip -> (y [Nb OH OW, Cout] bf16,
    part). epi 0; 5: part = [2, tiles, Cout] per-tile BatchNorm statistics of y; 8: y is a BatchNorm + ReLU output
    gradient, bias = that BatchNorm's input [Nb OH OW, Cout], z = its statistics, part = per-tile backward sums."""
    nb, h, w_, c = x.shape
    cout = w9.shape[0]
    oh, ow = (h + 2 * pad - 3) // stride + 1, (w_ + 2 * pad - 3) // stride + 1
    M = nb * oh * ow
    if cfg is None:
        cfg = gemm8_pick(M, cout, 9 * c)
    if cfg is None:
        raise ValueError(f"no gemm8 tile configuration for the {M}x{cout}x{9 * c} convolution")
    bm = gemm8_configs()[cfg][0]
    y = out if out is not None else torch.empty(M, cout, device=x.device, dtype=torch.bfloat16)
    part = torch.empty(2, M // bm, cout, device=x.device, dtype=torch.float32) if epi in (5, 8) else None
    b = None
    if epi == 8:
        b = bias.reshape(M, cout)
        if not (b.dtype == torch.bfloat16 and b.is_contiguous() and z is not None and z.dtype == torch.float32
                and z.numel() == 4 * cout and z.is_contiguous()):
            raise ValueError("gemm8_conv3x3 epi 8: need a contiguous bf16 [M, Cout] input and fp32 [4, Cout] stats")
    if not (x.is_contiguous() and w9.is_contiguous() and x.dtype == torch.bfloat16 and w9.dtype == torch.bfloat16):
        raise ValueError("gemm8_conv3x3: contiguous bf16 NHWC input and [Cout, 9 C] weight")
    check(_g8_fns()["conv"](int(cfg), int(epi), ptr(x), ptr(w9), ptr(b), ptr(y), ptr(z), ptr(part), nb, h, w_, c,
                            cout, stride, pad, stream_handle(x.device)), "mifx_gemm8_conv3x3")
    return y, part


def gemm8_nt_bnx(x2: torch.Tensor, w: torch.Tensor, ax: torch.Tensor, epi: int = 0, r: torch.Tensor | None = None,
                 cfg: int | None = None, out: torch.Tensor | None = None):
    """relu(x2 scale + shift) . w^T on csrc/gemm8.hip, the BatchNorm + ReLU applied to the X fragments in the kernel:
    x2 [M, K] bf16 (a BatchNorm's INPUT), w [N, K] bf16, ax fp32 [2, K] = (scale, shift) -> (Y [M, N] bf16, part). epi
    0; 5: part = per-tile BatchNorm statistics of Y; 6: Y += r ([M, N] bf16) with the statistics of the sum. K <= 2048."""
    M, K = x2.shape
    N = w.shape[0]
    if cfg is None:
        cfg = gemm8_pick(M, N, K, bnx=True)
    if cfg is None:
        raise ValueError(f"no gemm8 tile configuration for the {M}x{N}x{K} BatchNorm-operand product")
    if not (x2.is_contiguous() and w.is_contiguous() and x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and ax.dtype == torch.float32 and ax.is_contiguous() and ax.numel() == 2 * K):
        raise ValueError("gemm8_nt_bnx: contiguous bf16 x2 [M, K] / w [N, K] and fp32 [2, K] scale / shift")
    if epi == 6 and (r is None or not r.is_contiguous() or r.dtype != torch.bfloat16):
        raise ValueError("gemm8_nt_bnx epi 6: a contiguous bf16 [M, N] addend")
    bm = gemm8_configs()[cfg][0]
    y = out if out is not None else torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    part = torch.empty(2, M // bm, N, device=x2.device, dtype=torch.float32) if epi in (5, 6) else None
    check(_g8_fns()["nt_bnx"](int(cfg), int(epi), ptr(x2), ptr(w), ptr(r), ptr(y), ptr(part), M, N, K, ptr(ax),
                              stream_handle(x2.device)), "mifx_gemm8_nt_bnx")
    return y, part


def gemm8_nt(x2: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, epi: int = 0,
             cfg: int | None = None, z: torch.Tensor | None = None, out: torch.Tensor | None = None,
             r2: torch.Tensor | None = None):
    """x2 [M, K] bf16, w [N, K] bf16 -> (Y [M, N] bf16, aux). epi 0: X W^T; 1: + bias; 2: GELU(X W^T + bias), aux
    = Z = bf16(X W^T); 3: + bias as a bf16 [M, N] matrix; 4: dZ = (X W^T) o GELU'(z + bias), aux = per-tile column sums
    [M / BM, N] fp32; 5: aux = per-tile BatchNorm statistics of the stored Y, [2, M / BM, N] fp32 = (tile column mean,
    tile sum of squared deviations M2); 6: 3 and 5 (Y = X W^T + bias-matrix, statistics of the stored sum); 8: Y = X W^T
    is the output gradient of a BatchNorm + ReLU whose input is `bias` (bf16 [M, N]) and whose forward statistics are
    `z` (fp32 [4, N]: mean, rstd, scale, shift): aux = [2, M / BM, N] fp32 per-tile (sum g, sum g xhat) of its
    backward (csrc/bn_relu.hip mifx_bn_relu_bwd_tiles consumes them); 9: as 8 for Y = X W^T + r2 (bf16 [M, N])."""
    M, K = x2.shape
    N = w.shape[0]
    if cfg is None:
        cfg = gemm8_pick(M, N, K)
    if cfg is None:
        raise ValueError(f"no gemm8 tile configuration for {M}x{N}x{K}")
    bm = gemm8_configs()[cfg][0]
    x2, w = x2.contiguous(), w.contiguous()
    y = out if out is not None else torch.empty(M, N, device=x2.device, dtype=torch.bfloat16)
    aux, part = None, None
    b = None
    if epi == 2:
        z = aux = torch.empty_like(y)
    if epi in (3, 6):
        b = bias.reshape(M, N).to(torch.bfloat16).contiguous()
    elif epi in (1, 2, 4):
        b = bias if bias.dtype in (torch.float32, torch.bfloat16) else bias.float()
        b = b.contiguous()
    if epi == 4:
        part = aux = torch.empty(M // bm, N, device=x2.device, dtype=torch.float32)
    if epi in (5, 6, 8, 9):
        part = aux = torch.empty(2, M // bm, N, device=x2.device, dtype=torch.float32)
    if epi == 9:
        r2 = r2.reshape(M, N)
        if not (r2.dtype == torch.bfloat16 and r2.is_contiguous()):
            raise ValueError("gemm8_nt epi 9: r2 must be a contiguous bf16 [M, N] matrix")
    if epi in (8, 9):
        b = bias.reshape(M, N)
        if not (b.dtype == torch.bfloat16 and b.is_contiguous() and z is not None and z.dtype == torch.float32
                and z.numel() == 4 * N and z.is_contiguous()):
            raise ValueError("gemm8_nt epi 8: need a contiguous bf16 [M, N] input and fp32 [4, N] statistics")
    check(_g8_fns()["nt"](int(cfg), int(epi), int(b is not None and b.dtype == torch.float32), ptr(x2), ptr(w),
                          ptr(b), ptr(y), ptr(z), ptr(part), M, N, K, ptr(r2 if epi == 9 else None),
                          stream_handle(x2.device)), "mifx_gemm8_nt")
    return y, aux


# ---------------------------------------------------------------- exact fp32 GEMM with edge tiles (csrc/gemm_f32.hip)
@functools.lru_cache(maxsize=None)
def _f32_fns():
    lib = _lib.load("gemm_f32")
    return {"nn": sig(lib, "mifx_gemm_f32_nn", [VP, VP, VP, I32, I32, I32, I32, I32, I32, VP])}


def matmul_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a [M, K] @ b [K, N] in fp32 on the f32 matrix cores (exact fp32 products and accumulation), any shape:
    ragged edges are zero-filled in the kernel's tile loads. The KN18 anchor (the reference's 1000 x 1000 eager
    matmul) on a hand-written kernel; CPU tensors take torch.matmul."""
    if not a.is_cuda:
        return a @ b
    if a.dim() != 2 or b.dim() != 2 or a.shape[1] != b.shape[0] or a.dtype != torch.float32 or b.dtype != torch.float32:
        raise ValueError("matmul_f32 takes fp32 [M, K] and [K, N] CUDA tensors")
    a, b = a.contiguous(), b.contiguous()
    M, K = a.shape
    N = b.shape[1]
    c = torch.empty(M, N, device=a.device, dtype=torch.float32)
    native_stats.count("gemm_f32", True)
    check(_f32_fns()["nn"](ptr(a), ptr(b), ptr(c), M, N, K, K, N, N, stream_handle(a.device)), "mifx_gemm_f32_nn")
    return c


# ---------------------------------------------------------------- fused FFN block (BERT): one autograd node
# FFN-out's input gradient dH = dOut W2 and FFN-in's bias-GELU backward dZ = dH o GELU'(Z + b1) in ONE GEMM
# (csrc/gemm.hip EPI_GELU_BWD on the transposed W2 copy): the unfused path writes dH [tokens, 3072] and the
# bias_gelu backward kernel reads it back with Z. (M, N, K) of the dH GEMM -> NT configuration.
GELU_BWD_TUNED: dict[tuple[int, int, int], int] = {(4096, 3072, 768): 9}
_GELU_BWD_G8 = os.environ.get("MIFX_GELU_BWD_G8", "0") == "1"


def _gelu_bwd_gemm(dout2: torch.Tensor, w2: torch.Tensor, z: torch.Tensor, b1: torch.Tensor, cfg: int):
    """dZ = (dOut W2) o GELU'(Z + b1) and db1 = column sums of dZ: dout2 [M, K], w2 [K, N] (the FFN-out weight
    [out, in]), z [M, N] bf16."""
    M, K = dout2.shape
    N = w2.shape[1]
    bp = b1 if b1.dtype in (torch.float32, torch.bfloat16) else b1.float()
    if _GELU_BWD_G8:  # the pipelined kernel's GELU-backward epilogue (A/B: MIFX_GELU_BWD_G8=1)
        g8 = gemm8_pick(M, N, K)
        if g8 is not None:
            dz, part = gemm8_nt(dout2.contiguous(), transposed(w2), bp.contiguous(), 4, cfg=g8, z=z)
            from .fused_bert import col_sum

            return dz, col_sum(part, b1.dtype if b1.dtype in (torch.float32, torch.bfloat16) else torch.float32)
    bm = configs()[cfg][0]
    dz = torch.empty(M, N, device=dout2.device, dtype=torch.bfloat16)
    part = torch.empty(M // bm, N, device=dout2.device, dtype=torch.float32)
    check(_fns()["gelu_bwd"](int(cfg), int(bp.dtype == torch.float32), ptr(dout2.contiguous()), ptr(transposed(w2)),
                             ptr(bp.contiguous()), ptr(z), ptr(dz), ptr(part), M, N, K,
                             stream_handle(dout2.device)), "mifx_gemm_nt_gelu_bwd")
    from .fused_bert import col_sum

    return dz, col_sum(part, b1.dtype if b1.dtype in (torch.float32, torch.bfloat16) else torch.float32)


class _FFN(torch.autograd.Function):
    """out = GELU(x W1^T + b1) W2^T (no FFN-out bias: the caller fuses it into the next add + LayerNorm)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, slot=None, tp=None, tp_in=None):
        shp = x.shape
        ctx.tp_in = tp_in
        x2 = x.reshape(-1, shp[-1])
        from .fused_bert import _fns as fb_fns, _dt, _param

        if preferred(x2, w1):
            y1, z = fwd_nt(x2, w1, b1, 2)
        else:
            z = F.linear(x2, w1)
            bp = _param(b1)
            y1 = torch.empty_like(z)
            N = z.shape[-1]
            check(fb_fns()["gelu"](_dt(z), _dt(bp), 1, None, ptr(z), ptr(bp), z.numel() // N, N, ptr(y1), None,
                                   None, stream_handle(z.device)), "mifx_bert_bias_gelu")
        native_stats.count("gemm_fwd_bias_gelu", preferred(x2, w1))
        fwd2 = preferred(y1, w2)
        native_stats.count("gemm_fwd", fwd2)
        if tp is not None:  # row-parallel FFN-out: all-reduced here, overlapped with its GEMM chunk by chunk
            from ..parallel.tensor_parallel import gemm_allreduce_overlapped

            out = gemm_allreduce_overlapped(y1, lambda yc: gemm_nt(yc, w2)[0] if fwd2 else F.linear(yc, w2),
                                            w2.shape[0], tp)
        else:
            out = fwd_nt(y1, w2)[0] if fwd2 else F.linear(y1, w2)
        ctx.save_for_backward(x2, w1, b1, z, y1, w2)
        ctx.slot = slot
        return out.view(*shp[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dout):
        x2, w1, b1, z, y1, w2 = ctx.saved_tensors
        dout2 = dout.reshape(-1, dout.shape[-1]).to(y1.dtype).contiguous()
        dw2 = _dw(dout2, y1, w2)
        M, K = dout2.shape
        N = w2.shape[1]
        cfg = GELU_BWD_TUNED.get((M, N, K))
        if cfg is not None and os.environ.get("MIFX_HIP_GELU_BWD", "1") != "0":
            native_stats.count("gemm_dX_gelu_bwd", True)
            dz, db1 = _gelu_bwd_gemm(dout2, w2, z, b1, cfg)
        else:
            native_stats.count("gemm_dX_gelu_bwd", False)
            dh = _dx(dout2, w2, None)
            from .fused_bert import _fns as fb_fns, _dt, _param

            bp = _param(b1)
            dz = torch.empty_like(z)
            part = torch.empty(fb_fns()["gchunks"](M), N, device=z.device, dtype=torch.float32)
            db1 = torch.empty(N, device=z.device, dtype=bp.dtype)
            check(fb_fns()["gelu"](_dt(z), _dt(bp), 0, ptr(dh.to(z.dtype).contiguous()), ptr(z), ptr(bp), M, N,
                                   ptr(dz), ptr(part), ptr(db1), stream_handle(z.device)), "mifx_bert_bias_gelu")
        dw1 = _dw(dz, x2, w1)
        dx = _dx_reduced(dz, w1, ctx.slot, ctx.tp_in).view(*dout.shape[:-1], w1.shape[1]) \
            if ctx.needs_input_grad[0] else None
        return dx, dw1, db1.to(b1.dtype), dw2, None, None, None


def ffn(x: torch.Tensor, w1: torch.Tensor, b1: torch.Tensor, w2: torch.Tensor,
        slot: GradSlot | None = None, tp=None, tp_in=None) -> torch.Tensor:
    """GELU(x W1^T + b1) W2^T as one autograd node on the GPU (bf16): the FFN-out input gradient and the bias-GELU
    backward fused into one GEMM where tuned (GELU_BWD_TUNED); elsewhere the two-node composition. tp: FFN-out is
    row-parallel and its product comes back all-reduced (overlapped chunk by chunk); tp_in: x is replicated over the
    group (copy_to_tp folded in: the input gradient comes back all-reduced, overlapped with the dX GEMM)."""
    tin = tp_in if tp_in is not None and tp_in.size > 1 else None
    if x.is_cuda and x.dtype == torch.bfloat16 and w1.dtype == torch.bfloat16 and w2.dtype == torch.bfloat16:
        return _FFN.apply(x, w1, b1, w2, slot, tp, tin)
    if tin is not None:
        from ..parallel.tensor_parallel import copy_to_tp

        x = copy_to_tp(x, tin)
    return linear(linear_bias_gelu(x, w1, b1, slot=slot), w2)
