"""Inference form of ResNet-50 v2 (the TF-Hub `resnet_v2_50` serving model, 1 x 224 x 224 x 3 -> 1001
logits, pre-process /255, post-process argmax - 1; reference `notebooks/redis/utils/model_saver.py:1-14`,
`data_processing_script_tensorflow.py:1-9`).

In the pre-activation bottleneck every convolution but the last is followed by BatchNorm + ReLU. With the running
statistics frozen, that BatchNorm is a per-output-channel affine map, so it folds into the convolution:
w' = w * gamma / sqrt(var + eps) (per output channel), b' = beta - mean * gamma / sqrt(var + eps), and the ReLU runs in
the convolution's epilogue (csrc/gconv.hip forward: bias + ReLU) -- conv1 and conv2 of every block are ONE kernel
each, with no activation pass between them. The block-input BatchNorm + ReLU normalises the residual sum: one apply
kernel reads branch and shortcut and writes the sum (the next identity shortcut) and relu(bn(sum)) (csrc/bn_relu.hip
`mifx_bn_add_relu_apply`). (Running it in conv3's epilogue instead -- csrc/gconv.hip ResEpi, opt-in
MIFX_INFER_RES_EPI=1, bit-identical -- measured slower: 0.83 / 1.11 / 2.23 ms at B = 1 / 8 / 32 against 0.79 / 1.01 /
1.76, profiles/resnet_infer_resepi_r4.jsonl: the conv's store loop turns into a dependent load-add-store chain with
three times the traffic, on fewer workgroups than the standalone kernel.) At batch 1 the later stages have too few pixel x channel tiles for the chip, so their
convolutions split the reduction over workgroups (ordered fp32 partials). The 3-channel 7x7 stem stays on MIOpen (its
channel count does not tile the MFMA kernel). `graphed()` captures the whole forward for a fixed input shape in one
hipGraph.

Off the GPU (or for a shape the kernels do not take) the same folded weights run through F.conv2d, which is what
the CPU test checks the folding against."""
from __future__ import annotations

import functools
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import _lib, gconv
from ..ops._lib import I32, I64, VP, check, ptr, sig, stream_handle
from ..ops.pool import max_pool3s2
from .resnet import ResNetV2


_RES_EPI = os.environ.get("MIFX_INFER_RES_EPI", "0") == "1"  # residual + next BN in conv3's epilogue (see above)


@functools.lru_cache(maxsize=None)
def _bn_fns():
    lib = _lib.load("bn_relu")
    return sig(lib, "mifx_bn_add_relu_apply", [I32, VP, VP, VP, I64, I32, VP, VP, I32, VP])


def _affine(bn: nn.BatchNorm2d) -> tuple[torch.Tensor, torch.Tensor]:
    """Frozen BatchNorm as (scale, shift), fp32."""
    scale = bn.weight.detach().float() * torch.rsqrt(bn.running_var.detach().float() + bn.eps)
    shift = bn.bias.detach().float() - bn.running_mean.detach().float() * scale
    return scale.contiguous(), shift.contiguous()


class _FoldedConv:
    """A convolution with an optional frozen BatchNorm folded in (and ReLU after it)."""

    def __init__(self, conv: nn.Conv2d, bn: nn.BatchNorm2d | None, dtype: torch.dtype):
        w = conv.weight.detach().float()
        self.bias = None
        if bn is not None:
            scale, shift = _affine(bn)
            w = w * scale.view(-1, 1, 1, 1)
            self.bias = shift
        self.relu = bn is not None
        self.stride, self.pad = conv.stride[0], conv.padding[0]
        self.K, self.C, self.R, self.S = w.shape
        self.w = w.to(dtype).contiguous()  # [K, C, R, S] (the F.conv2d path)
        # the HIP kernel's layout [G = 1][K][R][S][C], bf16
        self.w_fwd = self.w.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous().view(1, self.K, self.R, self.S, self.C)

    def hip_ok(self, x: torch.Tensor) -> bool:
        return x.is_cuda and x.dtype == torch.bfloat16 and gconv.eligible(x, self.w, 1, self.pad, self.stride) \
            and x.is_contiguous(memory_format=torch.channels_last)

    def with_residual(self, x: torch.Tensor, res: torch.Tensor, scale2: torch.Tensor, shift2: torch.Tensor):
        """(s, relu(s * scale2 + shift2)) with s = this conv(x) + res: on the GPU one kernel (the conv's residual
        epilogue, csrc/gconv.hip ResEpi), else the separate ops."""
        if self.hip_ok(x) and not self.relu and res.dtype == torch.bfloat16 \
                and res.is_contiguous(memory_format=torch.channels_last):
            N, _, Hi, Wi = x.shape
            return gconv.launch_res(x, self.w_fwd, self.bias, N, Hi, Wi, 1, self.C, self.K, self.R, self.S, self.pad,
                                    self.stride, res, scale2, shift2)
        y, s = _bn_add_relu(self(x), res, scale2, shift2)
        return s, y

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if self.hip_ok(x):
            N, _, Hi, Wi = x.shape
            return gconv._launch(x, self.w_fwd, self.bias, N, Hi, Wi, 1, self.C, self.K, self.R, self.S, self.pad,
                                 self.relu, self.stride)
        y = F.conv2d(x, self.w.to(x.dtype), None if self.bias is None else self.bias.to(x.dtype), self.stride,
                     self.pad)
        return F.relu(y) if self.relu else y


def _bn_add_relu(a: torch.Tensor, b: torch.Tensor | None, scale: torch.Tensor, shift: torch.Tensor):
    """(relu(scale * s + shift), s) with s = a + b (b None: s = a): one kernel on channels-last GPU tensors."""
    native = a.is_cuda and a.dtype in (torch.bfloat16, torch.float32) and a.shape[1] % 8 == 0 \
        and a.is_contiguous(memory_format=torch.channels_last) \
        and (b is None or (b.dtype == a.dtype and b.shape == a.shape and b.is_contiguous(
            memory_format=torch.channels_last)))
    if native:
        N, C, H, W = a.shape
        y = torch.empty_like(a)
        s = torch.empty_like(a) if b is not None else a
        check(_bn_fns()(int(a.dtype == torch.bfloat16), ptr(a), ptr(b), ptr(s) if b is not None else None,
                        N * H * W, C, ptr(scale), ptr(shift), 1, ptr(y), stream_handle(a.device)),
              "mifx_bn_add_relu_apply")
        return y, s
    s = a if b is None else a + b
    y = torch.relu(s * scale.view(1, -1, 1, 1).to(s.dtype) + shift.view(1, -1, 1, 1).to(s.dtype))
    return y, s


class FoldedResNetV2:
    """Eval-mode ResNetV2 with its BatchNorms folded (see the module docstring). `__call__(x)`: x [B, 3, H, W] in
    [0, 1] (channels-last on the GPU) -> fp32 logits. Weights are copied at construction: re-fold after training."""

    def __init__(self, model: ResNetV2, dtype: torch.dtype | None = None):
        p = next(model.parameters())
        self.device = p.device
        self.dtype = dtype or (torch.bfloat16 if p.is_cuda else torch.float32)
        self.stem_w = model.stem.weight.detach().to(self.dtype).contiguous(memory_format=torch.channels_last) \
            if p.is_cuda else model.stem.weight.detach().to(self.dtype)
        self.blocks = []
        for blk in model.blocks:
            self.blocks.append({
                "bn0": _affine(blk.bn0),
                "sc": _FoldedConv(blk.shortcut, None, self.dtype) if blk.shortcut is not None else None,
                "c1": _FoldedConv(blk.conv1, blk.bn1, self.dtype),
                "c2": _FoldedConv(blk.conv2, blk.bn2, self.dtype),
                "c3": _FoldedConv(blk.conv3, None, self.dtype),
            })
        self.post = _affine(model.post_bn)
        self.fc_w = model.fc.weight.detach().float()
        self.fc_b = model.fc.bias.detach().float()

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        x = x.to(self.dtype)
        if x.is_cuda:
            x = x.contiguous(memory_format=torch.channels_last)
        y = max_pool3s2(F.conv2d(x, self.stem_w, None, 2, 3))
        pre, s = _bn_add_relu(y, None, *self.blocks[0]["bn0"])
        for i, b in enumerate(self.blocks):
            short = b["sc"](pre) if b["sc"] is not None else s
            # residual sum + the next BatchNorm + ReLU (the next block's, or the final one)
            nxt = self.blocks[i + 1]["bn0"] if i + 1 < len(self.blocks) else self.post
            h = b["c2"](b["c1"](pre))
            if _RES_EPI:
                s, pre = b["c3"].with_residual(h, short, *nxt)
            else:
                pre, s = _bn_add_relu(b["c3"](h), short, *nxt)
        return F.linear(pre.float().mean(dim=(2, 3)), self.fc_w, self.fc_b)

    def graphed(self, example: torch.Tensor):
        """The forward captured in one hipGraph for `example`'s shape: returns f(x) -> logits (a fresh tensor)."""
        static_in = example.detach().clone()
        if static_in.is_cuda:
            static_in = static_in.contiguous(memory_format=torch.channels_last)
        side = torch.cuda.Stream(static_in.device)
        side.wait_stream(torch.cuda.current_stream(static_in.device))
        with torch.cuda.stream(side):  # warm-up (library handles, MIOpen solution choice) outside the capture
            self(static_in)
        torch.cuda.current_stream(static_in.device).wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_out = self(static_in)

        def run(x: torch.Tensor) -> torch.Tensor:
            static_in.copy_(x)
            graph.replay()
            return static_out.clone()

        run.graph = graph
        return run
