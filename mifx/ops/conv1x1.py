"""1x1 convolutions of channels_last activations as GEMMs on the pipelined MFMA kernel, with the BatchNorm statistics
(and the residual add) folded into the epilogue (csrc/gemm8.hip EPI_STATS / EPI_ADD_STATS).

ResNet-50 v2 (BASELINE config 5) is pre-activation: conv1 (1x1) feeds BN1, and conv3 (1x1) plus the shortcut feeds the
next block's BN0. With MIOpen convolutions every such BatchNorm re-read its input for a statistics pass, and the
residual sum was recomputed by BN0's statistics AND apply passes (4 reads + 3 writes of the block output per block).
Here the GEMM that writes the activation also writes it ALREADY SUMMED with the residual and the per-tile (mean, M2)
of what it stored, so the BatchNorm only finalizes (a tiny kernel) and applies: 2 reads + 2 writes.

In NHWC a 1x1 stride-1 convolution is exactly Y[M, Cout] = X[M, Cin] W[Cout, Cin]^T with M = N H W. Backward:
dX = dY W on the same kernel against W^T where it tiles (Cin % 128), else MIOpen's backward-data convolution;
dW = dY^T X deferred into one grouped split-K launch of the pipelined TN kernel when inside
`mifx.ops.gemm.deferred_weight_grads()` (fp32, into .grad), else MIOpen's backward-weights -- and the residual's
gradient is dY itself.

When the input is the output of a BatchNorm + ReLU that feeds ONLY this convolution (`bn_input=True`: conv3 after BN2;
conv1 after BN0 in identity-shortcut blocks), the dX GEMM also reduces that BatchNorm's backward sums (sum g,
sum g xhat per tile, csrc/gemm8.hip EPI_BNBWD) and hands them to its node: the BatchNorm backward skips its own
reduction pass over dX and x (bn_relu.offer_bwd_tiles; it verifies the gradient it receives is that dX, unmodified)."""
from __future__ import annotations

import os

import torch

from . import gemm as hg
from . import native_stats, weight_prep
from ._lib import check, ptr, stream_handle

# dX backend for tileable shapes: "gemm8" (default) or "miopen" (A/B)
DGRAD = os.environ.get("MIFX_CONV1X1_DGRAD", "gemm8")


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1)


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] channels_last -> the [N H W, C] storage view."""
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def eligible(x: torch.Tensor, w: torch.Tensor, stride: int = 1) -> bool:
    """A stride-1 1x1 convolution the GEMM kernel tiles: bf16 channels_last CUDA input, Cout % 128, Cin % 64,
    N H W % 128."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and stride == 1 and w.dim() == 4
            and tuple(w.shape[2:]) == (1, 1) and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    n, cin, h, ww = x.shape
    return hg.gemm8_pick(n * h * ww, w.shape[0], cin) is not None


class _Conv1x1(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, r, stats, bn):
        cout, cin = w.shape[0], w.shape[1]
        im = weight_prep.images(w)  # this step's bf16 images (one launch for every convolution), else cast here
        wb = im[0] if im is not None else w.reshape(cout, cin).to(torch.bfloat16).contiguous()
        ctx.wt = im[1] if im is not None else None
        x2 = _rows(x)
        M = x2.shape[0]
        cfg = hg.gemm8_pick(M, cout, cin)
        out = torch.empty(x.shape[0], cout, x.shape[2], x.shape[3], device=x.device, dtype=torch.bfloat16,
                          memory_format=torch.channels_last)
        epi = (6 if r is not None else 5) if stats else (3 if r is not None else 0)
        rr = _rows(r.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)) if r is not None else None
        _, part = hg.gemm8_nt(x2, wb, rr, epi, cfg=cfg, out=_rows(out))
        ctx.save_for_backward(x2, wb)
        ctx.w = w
        ctx.has_r = r is not None
        ctx.shape = x.shape
        ctx.bn = bn
        if part is None:
            part = torch.empty(0, device=x.device)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.mark_non_differentiable(part)
        return out, part

    @staticmethod
    def backward(ctx, dy, dpart):
        x2, wb = ctx.saved_tensors
        if dy is None:
            return None, None, None, None, None
        dyc = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dy2 = _rows(dyc)
        w = ctx.w
        dw = None
        if ctx.needs_input_grad[1]:
            dw = hg.defer_weight_grad_f32(dy2, x2, w)
        want_dx, want_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1] and dw is None
        dx = None
        n, cin, h, w_ = ctx.shape
        cfg = hg.gemm8_pick(dy2.shape[0], cin, wb.shape[0]) if want_dx and DGRAD == "gemm8" else None
        if cfg is not None:
            dx = torch.empty(n, cin, h, w_, device=dy.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
            bn, xbn, stats = ctx.bn, None, None
            if bn is not None:
                xbn, _, stats = bn.saved_tensors
                if not (xbn.dtype == torch.bfloat16 and tuple(xbn.shape) == tuple(ctx.shape)
                        and xbn.is_contiguous(memory_format=torch.channels_last)):
                    xbn = None
            if xbn is not None:
                wt = ctx.wt if ctx.wt is not None else hg.transpose(wb)
                _, part = hg.gemm8_nt(dy2, wt, _rows(xbn), 8, cfg=cfg, z=stats, out=_rows(dx))
                from .bn_relu import offer_bwd_tiles
                offer_bwd_tiles(bn, dx, part)
            else:
                hg.gemm8_nt(dy2, ctx.wt if ctx.wt is not None else hg.transpose(wb), None, 0, cfg=cfg, out=_rows(dx))
            want_dx = False
        if want_dx or want_dw:
            # the input gradient (and a weight gradient the grouped flush does not take: Cin = 64) on MIOpen's NHWC
            # backward convolutions, one call: measured faster than the library GEMMs on these skinny products
            # (M = N H W up to 800k rows: hipBLASLt's dY^T X ran 1 ms on 16 workgroups)
            xin = x2.view(n, h, w_, cin).permute(0, 3, 1, 2)
            gx, gw, _ = torch.ops.aten.convolution_backward(dyc, xin, wb.view(wb.shape[0], cin, 1, 1), None, [1, 1],
                                                            [0, 0], [1, 1], False, [0, 0], 1,
                                                            [want_dx, want_dw, False])
            if want_dx:
                dx = gx
            if want_dw:
                native_stats.count("conv1x1_dW", False)
                dw = gw.to(w.dtype)
        return dx, dw, (dyc if ctx.has_r else None), None, None


def conv1x1(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor | None = None, stats: bool = False,
            bn_input: bool = False):
    """(conv2d(x, w) [+ residual], part): a 1x1 stride-1 convolution of a bf16 channels_last tensor on the GEMM
    kernel; with stats, part = [2, tiles, Cout] per-tile (mean, M2) of the stored output for
    BatchNormReLU2d.forward_tiles (else an empty tensor). bn_input: the caller guarantees x is a BatchNorm + ReLU
    output consumed by nothing else, so the input-gradient GEMM may reduce that BatchNorm's backward sums."""
    native_stats.count("conv1x1_fwd", True)
    bn = x.grad_fn if bn_input else None
    if bn is not None and not getattr(bn, "mifx_bn", False):
        bn = None
    return _Conv1x1.apply(x, w, residual, stats, bn)


# stride-2 1x1 shortcuts whose input gradient measured faster on the phase-split hand-written kernel,
# (input H, C, Cout) (profiles/resnet_conv_routes_r4.jsonl); others MIOpen
_HIP_DGRAD_S2 = {(56, 256, 512), (28, 512, 1024), (14, 1024, 2048)}
# the strided shortcut's forward and weight gradient on csrc/gemm8.hip (center-tap implicit GEMM, deferred grouped
# dW); MIFX_SC_G8=0 leaves both on MIOpen (A/B)
_SC_G8 = os.environ.get("MIFX_SC_G8", "1") != "0"


class _ProjPair(torch.autograd.Function):
    """A projection block's two consumers of the pre-activation: the strided 1x1 shortcut (forward: the center tap of
    the implicit-GEMM kernel; weight gradient: deferred into the grouped TN flush -- MIOpen's with MIFX_SC_G8=0; input
    gradient hand-written or MIOpen) and conv1 (the GEMM kernel with BN1's statistics in its
    epilogue), as ONE autograd node. Its backward computes the shortcut's input gradient first and hands it to conv1's
    input-gradient GEMM as the addend R2 (csrc/gemm8.hip EPI_ADD_BNBWD): the summed gradient of the pre-activation is
    written once -- no separate add of the two branches' gradients (autograd's, ~100 us each at B = 256) -- and, when
    the pre-activation is a BatchNorm + ReLU output feeding only this pair, the same epilogue reduces that BatchNorm's
    backward sums."""

    @staticmethod
    def forward(ctx, x, w_sc, w1, stride, bn):
        n, cin, h, w_ = x.shape
        c1, cs = w1.shape[0], w_sc.shape[0]
        oh, ow = (h - 1) // stride + 1, (w_ - 1) // stride + 1
        cfg_sc = hg.gemm8_pick(n * oh * ow, cs, cin) if _SC_G8 and cin >= 64 and not cin & (cin - 1) else None
        ctx.wtsc = None
        if stride == 1:  # (stage 1's projection) a plain GEMM over the same pixel rows as conv1
            im_sc = weight_prep.images(w_sc)
            wsc2 = im_sc[0] if im_sc is not None else w_sc.reshape(cs, cin).to(torch.bfloat16).contiguous()
            ctx.wtsc = im_sc[1] if im_sc is not None else None
            sc = torch.empty(n, cs, h, w_, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
            hg.gemm8_nt(_rows(x), wsc2, None, 0, cfg=hg.gemm8_pick(n * h * w_, cs, cin), out=_rows(sc))
            wsb = wsc2.view(cs, cin, 1, 1)
        elif cfg_sc is not None:  # the center tap of the implicit 3x3 GEMM: pixel (stride oh, stride ow)
            im_sc = weight_prep.images(w_sc)
            wsb = im_sc[0].view(cs, cin, 1, 1) if im_sc is not None else w_sc.to(torch.bfloat16)
            sc = torch.empty(n, cs, oh, ow, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
            hg.gemm8_conv1x1_strided(_nhwc(x), wsb.view(cs, cin), stride, 0, cfg=cfg_sc, out=_rows(sc))
        else:
            wsb = w_sc.to(torch.bfloat16)
            sc = torch.ops.aten.convolution(x, wsb, None, [stride, stride], [0, 0], [1, 1], False, [0, 0], 1)
        im = weight_prep.images(w1)
        wb1 = im[0] if im is not None else w1.reshape(c1, cin).to(torch.bfloat16).contiguous()
        ctx.wt1 = im[1] if im is not None else None
        x2 = _rows(x)
        y1 = torch.empty(n, c1, h, w_, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        _, part = hg.gemm8_nt(x2, wb1, None, 5, cfg=hg.gemm8_pick(x2.shape[0], c1, cin), out=_rows(y1))
        ctx.save_for_backward(x, wsb, wb1)
        ctx.w_sc, ctx.w1, ctx.stride, ctx.bn = w_sc, w1, stride, bn
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.mark_non_differentiable(part)
        return sc, y1, part

    @staticmethod
    def backward(ctx, dsc, dy1, dpart):
        x, wsb, wb1 = ctx.saved_tensors
        n, cin, h, w_ = x.shape
        stride = ctx.stride
        dx = dwsc = dw1 = None
        dx_sc = None
        if dsc is not None and stride == 1:
            dscc = dsc.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
            cs = wsb.shape[0]
            ds2 = _rows(dscc)
            if ctx.needs_input_grad[1]:
                dwsc = hg.defer_weight_grad_f32(ds2, _rows(x), ctx.w_sc)
                if dwsc is None:
                    dwsc = torch.ops.aten.convolution_backward(dscc, x, wsb, None, [1, 1], [0, 0], [1, 1], False,
                                                               [0, 0], 1, [False, True, False])[1].to(ctx.w_sc.dtype)
            if ctx.needs_input_grad[0]:  # the shortcut's input gradient: conv1's dX GEMM adds it (R2)
                wt = ctx.wtsc if ctx.wtsc is not None else hg.transpose(wsb.view(cs, cin))
                dx_sc = torch.empty(n, cin, h, w_, device=x.device, dtype=torch.bfloat16,
                                    memory_format=torch.channels_last)
                hg.gemm8_nt(ds2, wt, None, 0, cfg=hg.gemm8_pick(ds2.shape[0], cin, cs), out=_rows(dx_sc))
        elif dsc is not None:
            dscc = dsc.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
            cs = wsb.shape[0]
            if ctx.needs_input_grad[0] and (h, cin, cs) in _HIP_DGRAD_S2:
                from . import gconv

                dx_sc = gconv.dgrad_strided(dscc, wsb.contiguous(), n, h, w_, 1, cin, cs, 1, 1, 0, stride)
            want_dx = ctx.needs_input_grad[0] and dx_sc is None
            want_dw = ctx.needs_input_grad[1]
            if want_dw and _SC_G8:
                dwsc = hg.defer_strided1x1_weight_grad_f32(_rows(dscc), _nhwc(x), ctx.w_sc, stride)
                want_dw = dwsc is None
            if want_dx or want_dw:
                gx, gw, _ = torch.ops.aten.convolution_backward(dscc, x, wsb, None, [stride, stride], [0, 0], [1, 1],
                                                                False, [0, 0], 1, [want_dx, want_dw, False])
                if want_dx:
                    dx_sc = gx
                if want_dw:
                    dwsc = gw.to(ctx.w_sc.dtype)
        if dy1 is not None:
            dy1c = dy1.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
            dy2 = _rows(dy1c)
            x2 = _rows(x)
            if ctx.needs_input_grad[2]:
                dw1 = hg.defer_weight_grad_f32(dy2, x2, ctx.w1)
                if dw1 is None:
                    dw1 = torch.ops.aten.convolution_backward(dy1c, x, wb1.view(wb1.shape[0], cin, 1, 1), None, [1, 1],
                                                              [0, 0], [1, 1], False, [0, 0], 1,
                                                              [False, True, False])[1].to(ctx.w1.dtype)
            if ctx.needs_input_grad[0]:
                wt = ctx.wt1 if ctx.wt1 is not None else hg.transpose(wb1)
                cfg = hg.gemm8_pick(dy2.shape[0], cin, wb1.shape[0])
                dx = torch.empty(n, cin, h, w_, device=x.device, dtype=torch.bfloat16,
                                 memory_format=torch.channels_last)
                bn, xbn, stats = ctx.bn, None, None
                if bn is not None:
                    xbn, _, stats = bn.saved_tensors
                    if not (xbn.dtype == torch.bfloat16 and tuple(xbn.shape) == tuple(x.shape)
                            and xbn.is_contiguous(memory_format=torch.channels_last)):
                        xbn = None
                r2 = dx_sc.contiguous(memory_format=torch.channels_last) if dx_sc is not None else None
                if xbn is not None and r2 is not None:
                    _, part = hg.gemm8_nt(dy2, wt, _rows(xbn), 9, cfg=cfg, z=stats, out=_rows(dx), r2=_rows(r2))
                    from .bn_relu import offer_bwd_tiles

                    offer_bwd_tiles(bn, dx, part)
                elif r2 is not None:
                    hg.gemm8_nt(dy2, wt, _rows(r2), 3, cfg=cfg, out=_rows(dx))
                else:
                    hg.gemm8_nt(dy2, wt, None, 0, cfg=cfg, out=_rows(dx))
        elif ctx.needs_input_grad[0]:
            dx = dx_sc
        return dx, dwsc, dw1, None, None


# stride-1 projection shortcuts (ResNet-50 stage 1: 64 -> 256) in the pair too (MIFX_PAIR_S1=0: the separate node)
_PAIR_S1 = os.environ.get("MIFX_PAIR_S1", "1") != "0"


def proj_pair_eligible(x: torch.Tensor, w_sc: torch.Tensor, stride: int, w1: torch.Tensor) -> bool:
    """A 1x1 projection shortcut (strided, or stride 1 on the GEMM kernel both ways) and a GEMM-eligible 1x1 conv1
    on the same bf16 channels_last input."""
    if not (tuple(w_sc.shape[2:]) == (1, 1) and eligible(x, w1) and w_sc.shape[1] == x.shape[1]):
        return False
    if stride > 1:
        return True
    if not (_PAIR_S1 and stride == 1 and w_sc.shape[0] != x.shape[1]):
        return False
    m, cin, cs = x.shape[0] * x.shape[2] * x.shape[3], x.shape[1], w_sc.shape[0]
    return hg.gemm8_pick(m, cs, cin) is not None and hg.gemm8_pick(m, cin, cs) is not None


def proj_pair(x: torch.Tensor, w_sc: torch.Tensor, stride: int, w1: torch.Tensor, bn_input: bool = False):
    """(shortcut(x), conv1(x), conv1's per-tile BatchNorm statistics) as one node whose backward writes the summed
    input gradient once (see _ProjPair). bn_input: x is a BatchNorm + ReLU output consumed only by this pair."""
    native_stats.count("conv1x1_fwd", True)
    bn = x.grad_fn if bn_input else None
    if bn is not None and not getattr(bn, "mifx_bn", False):
        bn = None
    return _ProjPair.apply(x, w_sc, w1, int(stride), bn)


# BatchNorm + ReLU folded into the consumer 1x1 convolution: opt-in (MIFX_BN_FOLD=1). Same-box ResNet-50 A/B
# (profiles/resnet_bn_fold_ab_r5.txt): 11,954 vs 12,055 img/s without -- the forward apply passes it removes (~1.0 ms)
# are paid back by the re-derived activation write in the backward (~0.46 ms) and the AX GEMMs' smaller tiles (the
# 256 x 256 AX build spills registers: 128 x 128 runs conv3, +0.2 ms)
BN_FOLD = os.environ.get("MIFX_BN_FOLD", "0") == "1"


# weight gradient of a folded convolution from the grouped TN kernel's BatchNorm operand transform (MIFX_BNX_DW=1) or
# from the activation the BatchNorm backward re-derives (default)
_BNX_DW = os.environ.get("MIFX_BNX_DW", "0") == "1"


class _BNConv1x1(torch.autograd.Function):
    """relu(bn(x)) -> 1x1 convolution (+ residual) as ONE node whose activation is never stored: the forward finalizes
    the BatchNorm from the per-tile statistics of x (reduced by the GEMM that wrote x) and the convolution's GEMM
    applies relu(x scale + shift) to its X fragments as they leave LDS (csrc/gemm8.hip AX operands); the backward's
    input-gradient GEMM writes the activation's gradient with the BatchNorm's backward sums in its epilogue (EPI 8),
    the deferred weight gradient applies the same transform to its B operand (grouped TN BNX problems), and one
    finalize + apply pass gives dx (plus `dalias`: the gradient of the x alias output, e.g. the next identity
    shortcut's). Saves the BatchNorm's apply pass (a read and a write of the activation) in the forward."""

    @staticmethod
    def forward(ctx, x, part_in, gamma, beta, run_mean, run_var, momentum, eps, w, r):
        from . import bn_relu

        w32, stats = bn_relu._fwd_tiles(x, part_in, gamma, beta, run_mean, run_var, momentum, eps, True,
                                        apply=False)[1:]
        n, cin, h, w_ = x.shape
        cout = w.shape[0]
        im = weight_prep.images(w)
        wb = im[0] if im is not None else w.reshape(cout, cin).to(torch.bfloat16).contiguous()
        ctx.wt = im[1] if im is not None else None
        out = torch.empty(n, cout, h, w_, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        rr = _rows(r.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)) if r is not None else None
        _, part = hg.gemm8_nt_bnx(_rows(x), wb, stats[2:4], 6 if r is not None else 5, r=rr, out=_rows(out))
        ctx.save_for_backward(x, w32, stats, wb)
        ctx.w, ctx.has_r, ctx.wdtype = w, r is not None, gamma.dtype
        ctx.set_materialize_grads(False)
        ctx.mark_non_differentiable(part)
        return out, part, x.view_as(x)

    @staticmethod
    def backward(ctx, dout, dpart, dalias):
        from . import bn_relu

        x, w32, stats, wb = ctx.saved_tensors
        if dout is None:
            return (dalias, None, None, None) + (None,) * 6
        n, cin, h, w_ = x.shape
        cout = wb.shape[0]
        dyc = dout.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dy2 = _rows(dyc)
        x2 = _rows(x)
        wt = ctx.wt if ctx.wt is not None else hg.transpose(wb)
        dact = torch.empty(n, cin, h, w_, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        _, bpart = hg.gemm8_nt(dy2, wt, x2, 8, cfg=hg.gemm8_pick(dy2.shape[0], cin, cout), z=stats, out=_rows(dact))
        # the BatchNorm backward's apply pass reads x anyway: it also re-derives the activation for the weight
        # gradient (one extra write; the grouped TN kernel with the operand transform measured slower)
        want_dw = ctx.needs_input_grad[8]
        act = torch.empty_like(x) if want_dw and not _BNX_DW else None
        dx, dgb = bn_relu._bwd_tiles(dact, x, w32, stats, dalias, bpart, act=act)
        dw = None
        if want_dw:
            if act is not None:
                dw = hg.defer_weight_grad_f32(dy2, _rows(act), ctx.w)
            else:
                dw = hg.defer_weight_grad_f32(dy2, x2, ctx.w, bnx=stats[2:4])
            if dw is None:
                native_stats.count("conv1x1_dW", False)
                if act is None:
                    act = torch.empty_like(x)
                    check(bn_relu._fns()["apply"](1, ptr(x2), x2.shape[0], cin, ptr(stats[2]), ptr(stats[3]), 1,
                                                  ptr(_rows(act)), stream_handle(x.device)), "mifx_bn_relu_apply")
                dw = torch.ops.aten.convolution_backward(dyc, act, wb.view(cout, cin, 1, 1), None, [1, 1], [0, 0],
                                                         [1, 1], False, [0, 0], 1, [False, True, False])[1]
                dw = dw.to(ctx.w.dtype)
        return (dx, None, dgb[0].to(ctx.wdtype), dgb[1].to(ctx.wdtype), None, None, None, None, dw,
                dyc if ctx.has_r else None)


def bn_conv_eligible(x: torch.Tensor, part, bn, w: torch.Tensor) -> bool:
    """x (a BatchNorm + ReLU input with per-tile statistics `part`) -> 1x1 conv w foldable into one _BNConv1x1."""
    from . import bn_relu

    if not (BN_FOLD and part is not None and bn.training and bn.track_running_stats and bn_relu.native_ok(x)
            and x.dtype == torch.bfloat16 and eligible(x, w) and w.shape[1] == x.shape[1] and x.shape[1] <= 2048):
        return False
    n, cin, h, ww = x.shape
    M = n * h * ww
    return hg.gemm8_pick(M, w.shape[0], cin, bnx=True) is not None and hg.gemm8_pick(M, cin, w.shape[0]) is not None


def bn_conv1x1(x: torch.Tensor, part: torch.Tensor, bn, w: torch.Tensor, residual: torch.Tensor | None = None):
    """(conv1x1(relu(bn(x))) [+ residual], the output's per-tile statistics, x alias) with the activation never stored
    (see _BNConv1x1); bn: the BatchNormReLU2d (training, running statistics updated), part: x's per-tile statistics.
    Use the alias output where x itself is consumed again (an identity shortcut)."""
    native_stats.count("conv1x1_fwd", True)
    rm, rv, _ = bn._args()
    return _BNConv1x1.apply(x, part, bn.weight, bn.bias, rm, rv, bn.momentum, bn.eps, w, residual)
