"""3x3 convolutions of channels_last activations as implicit GEMMs on the pipelined MFMA kernel (csrc/gemm8.hip CV 1 /
CV 2), with the BatchNorm statistics of the output and the BatchNorm-backward sums of the input gradient in the
epilogues.

ResNet-50 v2's bottleneck conv2 (3x3, stride 1, or 2 in the first block of stages 2-4) sits between BN1 and BN2. On
MIOpen its forward, input gradient and weight gradient ran at ~13 % of the MFMA peak (the largest block of the step,
profiles/archive/resnet_steady_r5g.md) and BN2 / BN1 each needed a reduction pass. Here:

* forward: Y[Nb OH OW, Cout] = gathered X . W[Cout, 9 C]^T -- every 64-deep K-tile is one tap and a 64-channel slice,
  each gathered row one input pixel (or the zero page outside the image); the epilogue reduces BN2's per-tile
  (mean, M2) -- BatchNormReLU2d.forward_tiles then only finalizes and applies;
* input gradient (stride 1): the same kernel over dY with the flipped, transposed weight [C][3][3][Cout]; when the
  input is a BatchNorm + ReLU output consumed only by this convolution (`bn_input=True`), the epilogue also reduces
  that BatchNorm's backward sums (mifx.ops.conv1x1 does the same for 1x1). Stride 2: the phase-split hand-written
  kernel (mifx.ops.gconv.dgrad_strided) where it measured faster, else MIOpen;
* weight gradient: dW[Cout][3][3][C] = sum over output pixels of dY^T . X_tap, deferred into the grouped split-K TN
  launch with the 1x1 weight gradients (inside mifx.ops.gemm.deferred_weight_grads(), C and Cout % 256: 2048-pixel
  chunks of 256 x 256 tiles); the 64/128-channel ones on the nine-tap kernel of mifx.ops.conv3_wgrad (one staged input
  patch serves all taps; MIOpen's igemm_wrw before). Per-shape timings of every pass:
  profiles/conv3x3_routes_r5.jsonl (tools/bench_conv3x3.py).

Eligible: bf16 channels_last CUDA input, C a power of two >= 128 (>= 64: the narrow tiles; MIFX_CONV3X3_64=0 for >= 128),
Cout % 128 == 0 (% 64), padding 1, stride 1 or 2, and N OH OW a multiple of a tile height."""
from __future__ import annotations

import os

import torch

from . import gemm as hg
from . import conv3_wgrad, native_stats, weight_prep

# MIFX_CONV3X3=0 keeps the 3x3 convolutions on the routed MIOpen / gconv path (A/B); MIFX_CONV3X3_64=0 leaves
# the 64-channel ones (stage 1, on the narrow tiles: a tie with MIOpen in the step, profiles/resnet_narrow_ab_r5.txt)
ENABLED = os.environ.get("MIFX_CONV3X3", "1") != "0"
_SMALL = os.environ.get("MIFX_CONV3X3_64", "1") == "1"


# stride-2 input gradients where the phase-split hand-written kernel measured faster than MIOpen, (input H, C, Cout)
# (profiles/resnet_conv_routes_r4.jsonl); the others stay on MIOpen
_HIP_DGRAD_S2 = {(56, 128, 128), (28, 256, 256)}


def _rows(t: torch.Tensor) -> torch.Tensor:
    n, c, h, w = t.shape
    return t.permute(0, 2, 3, 1).reshape(n * h * w, c)


def _nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1)


def eligible(x: torch.Tensor, w: torch.Tensor, stride: int, padding: int) -> bool:
    if not (ENABLED and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and w.dim() == 4
            and tuple(w.shape[2:]) == (3, 3) and padding == 1 and stride in (1, 2)
            and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    n, c, h, w_ = x.shape
    cout = w.shape[0]
    if c < 64 or c & (c - 1) or cout % 64 or w.shape[1] != c or (stride == 1 and cout & (cout - 1)):
        return False  # (stride 1: the input gradient gathers dY, whose channel count must be a power of two too)
    if (c < 128 or cout < 128) and not _SMALL:
        return False
    oh, ow = (h + 2 - 3) // stride + 1, (w_ + 2 - 3) // stride + 1
    return hg.gemm8_pick(n * oh * ow, cout, 9 * c) is not None


def _w9(w: torch.Tensor) -> torch.Tensor:
    """[Cout, C, 3, 3] -> bf16 [Cout, 9 C] in (tap, channel) order (a channels_last weight's storage)."""
    wb = w.to(torch.bfloat16)
    return wb.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


class _Conv3x3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, stats, bn):
        n, c, h, w_ = x.shape
        cout = w.shape[0]
        oh, ow = (h - 1) // stride + 1, (w_ - 1) // stride + 1
        im = weight_prep.images(w)  # this step's bf16 images (one launch for every convolution), else cast here
        w9 = im[0] if im is not None else _w9(w)
        ctx.wt = im[1] if im is not None else None
        out = torch.empty(n, cout, oh, ow, device=x.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
        _, part = hg.gemm8_conv3x3(_nhwc(x), w9, stride, 1, epi=5 if stats else 0, out=_rows(out))
        ctx.save_for_backward(x, w9)
        ctx.w, ctx.stride, ctx.bn = w, stride, bn
        if part is None:
            part = torch.empty(0, device=x.device)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        ctx.mark_non_differentiable(part)
        return out, part

    @staticmethod
    def backward(ctx, dy, dpart):
        x, w9 = ctx.saved_tensors
        if dy is None:
            return None, None, None, None, None
        w, stride = ctx.w, ctx.stride
        n, c, h, w_ = x.shape
        cout = w9.shape[0]
        dyc = dy.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
        dy2 = _rows(dyc)
        dw = dx = None
        if ctx.needs_input_grad[1]:
            dw = hg.defer_conv3x3_weight_grad_f32(dy2, _nhwc(x), w, stride, 1)
            if dw is None and conv3_wgrad.eligible(x, dyc, w, stride):
                native_stats.count("conv3x3_dW", True)
                dw = conv3_wgrad.wgrad(x, dyc, w, stride)
            if dw is None:
                wb = w9.view(cout, 3, 3, c).permute(0, 3, 1, 2)
                native_stats.count("conv3x3_dW", False)
                dw = torch.ops.aten.convolution_backward(dyc, x, wb, None, [stride, stride], [1, 1], [1, 1], False,
                                                         [0, 0], 1, [False, True, False])[1].to(w.dtype)
        if ctx.needs_input_grad[0]:
            if stride == 1:
                # dX = conv(dY, W flipped and transposed): [C][3][3][Cout], the same implicit GEMM over dY's pixels
                wt = ctx.wt if ctx.wt is not None else \
                    w9.view(cout, 3, 3, c).flip(1, 2).permute(3, 1, 2, 0).reshape(c, 9 * cout).contiguous()
                dx = torch.empty(n, c, h, w_, device=dy.device, dtype=torch.bfloat16,
                                 memory_format=torch.channels_last)
                bn, xbn, stats = ctx.bn, None, None
                if bn is not None:
                    xbn, _, stats = bn.saved_tensors
                    if not (xbn.dtype == torch.bfloat16 and tuple(xbn.shape) == tuple(x.shape)
                            and xbn.is_contiguous(memory_format=torch.channels_last)):
                        xbn = None
                if xbn is not None:
                    _, part = hg.gemm8_conv3x3(_nhwc(dyc), wt, 1, 1, epi=8, bias=_rows(xbn), z=stats, out=_rows(dx))
                    from .bn_relu import offer_bwd_tiles

                    offer_bwd_tiles(bn, dx, part)
                else:
                    hg.gemm8_conv3x3(_nhwc(dyc), wt, 1, 1, epi=0, out=_rows(dx))
            elif (h, c, cout) in _HIP_DGRAD_S2:
                from . import gconv

                wb = w9.view(cout, 3, 3, c).permute(0, 3, 1, 2).contiguous()
                dx = gconv.dgrad_strided(dyc, wb, n, h, w_, 1, c, cout, 3, 3, 1, stride)
            else:
                wb = w9.view(cout, 3, 3, c).permute(0, 3, 1, 2)
                dx = torch.ops.aten.convolution_backward(dyc, x, wb, None, [stride, stride], [1, 1], [1, 1], False,
                                                         [0, 0], 1, [True, False, False])[0]
        return dx, dw, None, None, None


def conv3x3(x: torch.Tensor, w: torch.Tensor, stride: int = 1, stats: bool = False, bn_input: bool = False):
    """(conv2d(x, w, stride, padding 1), part) on the implicit-GEMM kernel (eligible() inputs); with stats, part =
    [2, tiles, Cout] per-tile (mean, M2) of the output for BatchNormReLU2d.forward_tiles (else empty). bn_input: x is a
    BatchNorm + ReLU output consumed by nothing else (its backward sums then come from the dX epilogue, stride 1)."""
    native_stats.count("conv3x3_fwd", True)
    bn = x.grad_fn if bn_input and stride == 1 else None
    if bn is not None and not getattr(bn, "mifx_bn", False):
        bn = None
    return _Conv3x3.apply(x, w, int(stride), bool(stats), bn)
