"""Grouped stride-1 NHWC convolution on hand-written bf16 MFMA implicit-GEMM kernels (csrc/gconv.hip).

`conv2d(x, weight, bias, padding, groups, stride=...)` == `F.conv2d(...)` for channels-last bf16 activations: the
forward and the stride-1 input gradient run one HIP kernel (the input gradient of a stride-1 conv is the same
kernel on dy with the weight flipped and transposed), a strided conv's input gradient a phase-split kernel
(`dgrad_strided`), the weight gradient a third one (transposed LDS reads). `eligible()` says when a call can take this path
(GPU, C/group % 32 == 0, K/group % 32 == 0 (the input gradient likewise, with the roles of C and K swapped); the weight
gradient needs C/group % 8 == 0 and splits over output pixels when there are few (tap, k, group) tiles); otherwise callers use F.conv2d. SURVEY KN14; used by the PATE teacher
ensemble (`mifx/privacy/pate/ensemble.py`)."""
from __future__ import annotations

import functools

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("gconv")
    return {"fwd": sig(lib, "mifx_gconv_fwd", [VP, VP, VP, VP] + [I32] * 11 + [VP]),
            "fwd_sk": sig(lib, "mifx_gconv_fwd_splitk", [VP, VP, VP, VP] + [I32] * 11 + [VP, I32, VP]),
            "ksplit": sig(lib, "mifx_gconv_fwd_ksplit", [I32] * 10),
            "fwd_ex": sig(lib, "mifx_gconv_fwd_ex", [VP, VP, VP, VP] + [I32] * 11 + [VP, I32, VP, VP, VP, VP, VP]),
            "wgrad": sig(lib, "mifx_gconv_wgrad", [VP, VP, VP] + [I32] * 11 + [VP, VP]),
            "wsplits": sig(lib, "mifx_gconv_wgrad_splits", [I32] * 10),
            "dgrad_s": sig(lib, "mifx_gconv_dgrad_strided", [VP, VP, VP] + [I32] * 10 + [VP])}


def dgrad_strided(dyb: torch.Tensor, wb: torch.Tensor, N, Hi, Wi, G, C, K, R, S, pad, stride) -> torch.Tensor:
    """Input gradient of a strided (grouped) convolution on the phase-split HIP kernel: dy bf16 channels-last
    [N, G*K, Ho, Wo], weight bf16 [G*K, C, R, S] -> dx bf16 channels-last [N, G*C, Hi, Wi]."""
    wt = wb.view(G, K, C, R, S).permute(0, 2, 3, 4, 1).contiguous()  # [G][C][R][S][K], not flipped
    dx = torch.empty(N, G * C, Hi, Wi, device=dyb.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
    check(_fns()["dgrad_s"](ptr(dyb), ptr(wt), ptr(dx), N, Hi, Wi, G, C, K, R, S, pad, int(stride),
                            stream_handle(dyb.device)), "mifx_gconv_dgrad_strided")
    return dx


def eligible(x: torch.Tensor, weight: torch.Tensor, groups: int, padding: int, stride: int = 1) -> bool:
    if not (x.is_cuda and x.dim() == 4 and weight.dim() == 4):
        return False
    GK, C, R, S = weight.shape
    if x.shape[1] != C * groups or GK % groups:
        return False
    K = GK // groups
    Ho, Wo = x.shape[2] + 2 * padding - R + 1, x.shape[3] + 2 * padding - S + 1
    return stride >= 1 and C % 32 == 0 and K % 32 == 0 and Ho > 0 and Wo > 0 and 0 <= padding < min(R, S)


def launch_res(x_nhwc: torch.Tensor, w_gkrsc: torch.Tensor, bias, N, Hi, Wi, G, C, K, R, S, pad, stride: int,
               res: torch.Tensor, scale2: torch.Tensor, shift2: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """Forward conv with the residual epilogue (inference of a pre-activation block): s = conv(x) (+ bias) + res,
    y2 = relu(s * scale2 + shift2) -- the residual sum and the next block's BatchNorm + ReLU in the conv's epilogue,
    rounded as the separate kernels round them. res: bf16 channels-last like the output; scale2 / shift2 fp32 [G*K].
    Returns (s, y2)."""
    Ho, Wo = (Hi + 2 * pad - R) // stride + 1, (Wi + 2 * pad - S) // stride + 1
    if tuple(res.shape) != (N, G * K, Ho, Wo) or res.dtype != torch.bfloat16 or \
            not res.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("residual must be a bf16 channels-last tensor shaped like the output")
    y = torch.empty(N, G * K, Ho, Wo, device=x_nhwc.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
    y2 = torch.empty_like(y)
    ks = int(_fns()["ksplit"](N, Hi, Wi, G, C, K, R, S, pad, int(stride)))
    part = torch.empty(ks * N * Ho * Wo * G * K, device=x_nhwc.device, dtype=torch.float32) if ks > 1 else None
    check(_fns()["fwd_ex"](ptr(x_nhwc), ptr(w_gkrsc), ptr(bias), ptr(y), N, Hi, Wi, G, C, K, R, S, pad, int(stride), 0,
                           ptr(part), ks, ptr(res), ptr(scale2), ptr(shift2), ptr(y2), stream_handle(x_nhwc.device)),
          "mifx_gconv_fwd_ex")
    return y, y2


def _launch(x_nhwc: torch.Tensor, w_gkrsc: torch.Tensor, bias, N, Hi, Wi, G, C, K, R, S, pad,
            relu: bool = False, stride: int = 1) -> torch.Tensor:
    Ho, Wo = (Hi + 2 * pad - R) // stride + 1, (Wi + 2 * pad - S) // stride + 1
    y = torch.empty(N, G * K, Ho, Wo, device=x_nhwc.device, dtype=torch.bfloat16, memory_format=torch.channels_last)
    # few pixel x channel tiles (batch-1 inference): the reduction split over workgroups, fp32 partials summed in
    # order by a second kernel (csrc/gconv.hip gconv_splitk_finish)
    ks = int(_fns()["ksplit"](N, Hi, Wi, G, C, K, R, S, pad, int(stride)))
    part = torch.empty(ks * N * Ho * Wo * G * K, device=x_nhwc.device, dtype=torch.float32) if ks > 1 else None
    check(_fns()["fwd_sk"](ptr(x_nhwc), ptr(w_gkrsc), ptr(bias), ptr(y), N, Hi, Wi, G, C, K, R, S, pad, int(stride),
                           int(relu), ptr(part), ks, stream_handle(x_nhwc.device)), "mifx_gconv_fwd")
    return y


WGRAD_HIP_SINGLE_GROUP = False  # single-group weight gradients on the HIP kernel too (A/B switch)


def wgrad(xb: torch.Tensor, dyb: torch.Tensor, N, Hi, Wi, G, C, K, R, S, pad, stride) -> torch.Tensor:
    """Weight gradient [G*K, C, R, S] fp32 of a (grouped, strided) conv on the HIP kernel: x / dy bf16
    channels-last; split over output pixels when the (tap, k, group) tiles alone cannot fill the chip."""
    sp = int(_fns()["wsplits"](N, Hi, Wi, G, C, K, R, S, pad, int(stride)))
    dw = torch.empty(G * K, C, R, S, device=dyb.device, dtype=torch.float32)
    part = torch.empty(sp * dw.numel(), device=dyb.device, dtype=torch.float32) if sp > 1 else None
    check(_fns()["wgrad"](ptr(xb), ptr(dyb), ptr(dw), N, Hi, Wi, G, C, K, R, S, pad, int(stride), sp, ptr(part),
                          stream_handle(dyb.device)), "mifx_gconv_wgrad")
    return dw


def _lib_bwd(xb, wb, dyb, stride: int, pad: int, groups: int, dgrad: bool, wgrad: bool):
    """MIOpen's backward through the op autograd itself uses (aten.convolution_backward): torch.nn.grad.conv2d_input
    / conv2d_weight take a different, much slower path on channels-last bf16 (4x on ResNet-50's input gradients,
    profiles/resnet_conv_routes_r4.jsonl)."""
    dx, dw, _ = torch.ops.aten.convolution_backward(dyb, xb, wb, None, [stride, stride], [pad, pad], [1, 1], False,
                                                    [0, 0], groups, [dgrad, wgrad, False])
    return dx, dw


class _GConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, pad, groups, relu, stride, route=None):
        N, _, Hi, Wi = x.shape
        GK, C, R, S = weight.shape
        G, K = groups, GK // groups
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wb = weight.to(torch.bfloat16)
        w_fwd = wb.view(G, K, C, R, S).permute(0, 1, 3, 4, 2).contiguous()  # [G][K][R][S][C]
        b = bias.float().contiguous() if bias is not None else None
        y = _launch(xb, w_fwd, b, N, Hi, Wi, G, C, K, R, S, pad, relu, stride)
        ctx.save_for_backward(xb, wb, y if relu else None)
        ctx.geo = (N, Hi, Wi, G, C, K, R, S, pad, bias is not None, weight.dtype,
                   bias.dtype if bias is not None else None, stride)
        ctx.route = route or (None, None)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wb, y = ctx.saved_tensors
        N, Hi, Wi, G, C, K, R, S, pad, has_bias, wdt, bdt, stride = ctx.geo
        dyb = dy.to(torch.bfloat16)
        if y is not None:  # fused ReLU: gradient through max(., 0)
            dyb = torch.ops.aten.threshold_backward(dyb, y, 0)
        dyb = dyb.contiguous(memory_format=torch.channels_last)
        Ho, Wo = dyb.shape[2], dyb.shape[3]
        dx = dw = db = None
        M = N * Ho * Wo
        r_dgrad, r_wgrad = ctx.route
        if ctx.needs_input_grad[0]:
            # HIP input gradient for grouped / large-image convs; MIOpen's is as fast or faster on small
            # single-group images (profiles/archive/gconv_resnet_r2.jsonl); a per-shape route overrides the policy
            hip_ok = C % 32 == 0 and K % 32 == 0 and R == S
            if r_dgrad == "miopen" or (r_dgrad == "hip" and not hip_ok):
                dx = _lib_bwd(xb, wb, dyb, stride, pad, G, True, False)[0]
            elif stride == 1 and C % 32 == 0 and R == S and (G > 1 or M >= 100_000 or r_dgrad == "hip"):
                # dx = conv(dy, flip(w) transposed), pad' = R - 1 - pad: [G][C][R][S][K] weight image
                w_bwd = wb.view(G, K, C, R, S).flip(3, 4).permute(0, 2, 3, 4, 1).contiguous()
                dx = _launch(dyb, w_bwd, None, N, Ho, Wo, G, K, C, R, S, R - 1 - pad)
            elif stride > 1 and C % 32 == 0 and K % 32 == 0:  # phase-split strided input gradient
                dx = dgrad_strided(dyb, wb, N, Hi, Wi, G, C, K, R, S, pad, stride)
            else:
                dx = _lib_bwd(xb, wb, dyb, stride, pad, G, True, False)[0]
        if ctx.needs_input_grad[1]:
            # Weight-gradient policy from measurements (profiles/archive/gconv_resnet_shapes_r3.jsonl,
            # pate_ensemble_bench_r3*.jsonl): grouped 1x1 -> one batched GEMM; other grouped convs -> the HIP kernel;
            # a single group (ResNet-50) -> MIOpen, which beats the pixel-split kernel on 7 of the 9 ResNet shapes.
            one_by_one = R == 1 and S == 1 and pad == 0 and stride == 1
            if r_wgrad == "miopen" or (r_wgrad == "hip" and not (C % 8 == 0 and K % 8 == 0)):
                dw = _lib_bwd(xb, wb, dyb, stride, pad, G, False, True)[1].to(wdt)
            elif r_wgrad == "hip":
                dw = wgrad(xb, dyb, N, Hi, Wi, G, C, K, R, S, pad, stride).to(wdt)
            elif G > 1 and one_by_one:  # dw[g] = dy_g^T x_g, one strided batched GEMM (no copies)
                dyv = dyb.permute(0, 2, 3, 1).reshape(M, G, K).permute(1, 2, 0)
                xv = xb.permute(0, 2, 3, 1).reshape(M, G, C).permute(1, 0, 2)
                dw = torch.bmm(dyv, xv, out_dtype=torch.float32).reshape(G * K, C, 1, 1).to(wdt)
            elif (G > 1 or WGRAD_HIP_SINGLE_GROUP) and C % 8 == 0 and K % 8 == 0:
                # hand-written weight gradient (fp32 out, PyTorch layout), split over output pixels when the
                # (tap, k, group) tiles alone cannot fill the chip (deterministic split sum)
                dw = wgrad(xb, dyb, N, Hi, Wi, G, C, K, R, S, pad, stride).to(wdt)
            else:
                dw = _lib_bwd(xb, wb, dyb, stride, pad, G, False, True)[1].to(wdt)
        if has_bias and ctx.needs_input_grad[2]:
            db = torch.sum(dyb, dim=(0, 2, 3), dtype=torch.float32).to(bdt)
        return dx, dw, db, None, None, None, None, None


class _LibFwdHipDgrad(torch.autograd.Function):
    """Single-group convolution with MIOpen's forward and weight gradient and the hand-written input gradient (the
    per-shape route where only the input gradient measured faster: profiles/resnet_conv_routes_r4.jsonl)."""

    @staticmethod
    def forward(ctx, x, weight, pad, stride):
        xb = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wb = weight.to(torch.bfloat16)
        y = torch.ops.aten.convolution(xb, wb, None, [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1)
        ctx.save_for_backward(xb, wb)
        ctx.geo = (pad, stride, weight.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wb = ctx.saved_tensors
        pad, stride, wdt = ctx.geo
        N, C, Hi, Wi = xb.shape
        K, _, R, S = wb.shape
        dyb = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            if stride == 1:
                w_bwd = wb.view(1, K, C, R, S).flip(3, 4).permute(0, 2, 3, 4, 1).contiguous()
                dx = _launch(dyb, w_bwd, None, N, dyb.shape[2], dyb.shape[3], 1, K, C, R, S, R - 1 - pad)
            else:
                dx = dgrad_strided(dyb, wb, N, Hi, Wi, 1, C, K, R, S, pad, stride)
        if ctx.needs_input_grad[1]:
            dw = _lib_bwd(xb, wb, dyb, stride, pad, 1, False, True)[1].to(wdt)
        return dx, dw, None, None


def conv2d_hip_dgrad(x: torch.Tensor, weight: torch.Tensor, padding: int, stride: int) -> torch.Tensor:
    """MIOpen forward / weight gradient, hand-written input gradient (single group, C and K % 32, square kernel)."""
    K, C, R, S = weight.shape
    if x.is_cuda and C % 32 == 0 and K % 32 == 0 and R == S and 0 <= padding < R and _lib.gpu_available():
        return _LibFwdHipDgrad.apply(x, weight, int(padding), int(stride))
    return F.conv2d(x, weight, None, stride=stride, padding=padding)


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor | None = None, padding: int = 0,
           groups: int = 1, relu: bool = False, stride: int = 1, route: tuple | None = None) -> torch.Tensor:
    """(Grouped, strided) convolution (`relu=True`: followed by ReLU, fused into the kernel's epilogue); the HIP
    kernels when `eligible`, else F.conv2d. Output bf16 channels-last on the kernel path (the dtype F.conv2d gives
    under bf16 autocast). route = (input-gradient backend, weight-gradient backend), each "hip", "miopen" or None
    (the built-in policy): a per-shape choice from measurements (mifx.models.resnet.CONV_ROUTES)."""
    if eligible(x, weight, groups, padding, stride) and _lib.gpu_available():
        return _GConv.apply(x, weight, bias, int(padding), int(groups), bool(relu), int(stride), route)
    y = F.conv2d(x, weight, bias, stride=stride, padding=padding, groups=groups)
    return F.relu(y) if relu else y
