"""ResNet-50 v2 (pre-activation) image classifier, 1001 classes (TF-Hub `resnet_v2_50` layout used by
the RedisAI demo, `notebooks/redis/utils/model_saver.py:1-14`; KN17). Channels-last so MIOpen runs
its NHWC MFMA convolutions; `inference_mode` + bf16 autocast for serving."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

import os

from ..ops.stem import eligible as stem_eligible, stem_conv
from ..ops import gconv
from ..ops.bn_relu import BatchNormReLU2d
from ..ops.pool import max_pool3s2

# Convolution backends (MIFX_RESNET_HIP_CONV): "routed" -- per shape and pass, the faster of the hand-written MFMA
# implicit-GEMM kernels (csrc/gconv.hip: forward, stride-1 / phase-split strided input gradient, pixel-split weight
# gradient) and MIOpen, from the measurement of every ResNet-50 convolution at B = 256 (CONV_ROUTES below,
# tools/bench_resnet_convs.py; the default: 25.8 vs 26.2 ms per step at B = 256, profiles/resnet_routed_ab_r4.txt);
# "1" -- every eligible pass on the HIP kernels (gconv's own policy); "0" -- MIOpen.
_MODE = os.environ.get("MIFX_RESNET_HIP_CONV", "routed")
USE_HIP_CONV = _MODE != "0"

# (input H, C in, K out, kernel, stride) -> (forward, input gradient, weight gradient) backend, measured per pass at
# B = 256 with MIOpen through aten.convolution_backward (profiles/resnet_conv_routes_r4.jsonl): MIOpen's forward and
# weight gradient win on every shape; the hand-written input gradient wins on the 17 shapes below (0.55 ms of the
# 17.9 ms of convolution per step). Shapes not listed (and the 3-channel stem) stay on MIOpen.
CONV_ROUTES: dict[tuple[int, int, int, int, int], tuple[str, str, str]] = {
    (7, 2048, 512, 1, 1): ('miopen', 'hip', 'miopen'),
    (14, 1024, 256, 1, 1): ('miopen', 'hip', 'miopen'),
    (14, 1024, 512, 1, 1): ('miopen', 'hip', 'miopen'),
    (14, 1024, 2048, 1, 2): ('miopen', 'hip', 'miopen'),
    (28, 128, 128, 3, 1): ('miopen', 'hip', 'miopen'),
    (28, 128, 512, 1, 1): ('miopen', 'hip', 'miopen'),
    (28, 256, 256, 3, 2): ('miopen', 'hip', 'miopen'),
    (28, 512, 128, 1, 1): ('miopen', 'hip', 'miopen'),
    (28, 512, 256, 1, 1): ('miopen', 'hip', 'miopen'),
    (28, 512, 1024, 1, 2): ('miopen', 'hip', 'miopen'),
    (56, 64, 64, 1, 1): ('miopen', 'hip', 'miopen'),
    (56, 64, 64, 3, 1): ('miopen', 'hip', 'miopen'),
    (56, 64, 256, 1, 1): ('miopen', 'hip', 'miopen'),
    (56, 128, 128, 3, 2): ('miopen', 'hip', 'miopen'),
    (56, 256, 64, 1, 1): ('miopen', 'hip', 'miopen'),
    (56, 256, 128, 1, 1): ('miopen', 'hip', 'miopen'),
    (56, 256, 512, 1, 2): ('miopen', 'hip', 'miopen'),
}


class HipConv2d(nn.Conv2d):
    """nn.Conv2d whose CUDA forward / backward run csrc/gconv.hip when the shape is eligible (channels % 32,
    symmetric padding < kernel) and routed there; bf16 channels-last output like F.conv2d under bf16 autocast."""

    def forward(self, x):
        if x.is_cuda and self.groups == 1 and self.dilation == (1, 1) and self.padding[0] == self.padding[1] \
                and self.stride[0] == self.stride[1] and self.kernel_size[0] == self.kernel_size[1] \
                and gconv.eligible(x, self.weight, 1, self.padding[0], self.stride[0]):
            route = None
            if _MODE == "routed":
                r = CONV_ROUTES.get((x.shape[2], self.in_channels, self.out_channels, self.kernel_size[0],
                                     self.stride[0]))
                if r is None or "hip" not in r:
                    return super().forward(x)
                if r[0] != "hip":  # MIOpen forward / weight gradient, hand-written input gradient
                    return gconv.conv2d_hip_dgrad(x, self.weight, self.padding[0], self.stride[0])
                route = (r[1], r[2])
            return gconv.conv2d(x, self.weight, self.bias, padding=self.padding[0], stride=self.stride[0],
                                route=route)
        return super().forward(x)


def _conv(*a, **kw):
    return (HipConv2d if USE_HIP_CONV else nn.Conv2d)(*a, **kw)


# Stride-1 1x1 convolutions as GEMMs on csrc/gemm8.hip with the BatchNorm statistics -- and for conv3 the residual
# add -- in the epilogue (mifx.ops.conv1x1): conv1 -> BN1 needs no statistics pass; conv3 + shortcut is written ALREADY
# SUMMED with the per-tile statistics of the sum, which the next block's BN0 only finalizes and applies.
# MIFX_RESNET_FUSED_1X1=0 keeps every convolution on the routed MIOpen / gconv path.
FUSED_1X1 = os.environ.get("MIFX_RESNET_FUSED_1X1", "1") != "0"


class Fused:
    """A block output already summed with its shortcut, with the per-tile BatchNorm statistics of the sum."""

    __slots__ = ("t", "part")

    def __init__(self, t, part):
        self.t, self.part = t, part


def _fused_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    from ..ops import conv1x1

    return FUSED_1X1 and conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.bias is None \
        and conv.groups == 1 and conv1x1.eligible(x, conv.weight)


def _fused3_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    from ..ops import conv3x3

    return FUSED_1X1 and conv.kernel_size == (3, 3) and conv.padding == (1, 1) and conv.bias is None \
        and conv.groups == 1 and conv.stride[0] == conv.stride[1] and conv.dilation == (1, 1) \
        and conv3x3.eligible(x, conv.weight, conv.stride[0], 1)


class _GlobalAvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shape, ctx.cl = x.shape, x.is_contiguous(memory_format=torch.channels_last)
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, dy):
        n, c, h, w = ctx.shape
        fmt = torch.channels_last if ctx.cl else torch.contiguous_format
        dx = torch.empty(n, c, h, w, device=dy.device, dtype=dy.dtype, memory_format=fmt)
        dx.copy_((dy * (1.0 / (h * w)))[:, :, None, None].expand(n, c, h, w))  # one pass in dx's own layout
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """x.mean((2, 3)) ([N, C]) whose gradient keeps x's memory format."""
    return _GlobalAvgPool.apply(x)


class PreActBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int):
        super().__init__()
        cout = width * self.expansion
        self.bn0 = BatchNormReLU2d(cin)  # every BN of the pre-activation net feeds a ReLU: fused
        self.shortcut = _conv(cin, cout, 1, stride=stride, bias=False) if (stride != 1 or cin != cout) else None
        self.conv1 = _conv(cin, width, 1, bias=False)
        self.bn1 = BatchNormReLU2d(width)
        self.conv2 = _conv(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormReLU2d(width)
        self.conv3 = _conv(width, cout, 1, bias=False)

    def forward(self, x):
        """x: a tensor, the (branch, shortcut) pair of the previous block whose sum is this block's input -- the
        residual add then happens inside bn0's fused kernels (fwd and bwd) -- or a `Fused` sum whose statistics the
        producing GEMM already reduced. Returns the un-added (branch, shortcut) pair, or a `Fused` sum when conv3 ran
        on the GEMM kernel, for the next block / the final BN."""
        from ..ops.conv1x1 import bn_conv1x1, bn_conv_eligible, conv1x1, proj_pair, proj_pair_eligible
        from ..ops.conv3x3 import conv3x3

        h = None
        if isinstance(x, Fused) and self.shortcut is None and bn_conv_eligible(x.t, x.part, self.bn0,
                                                                               self.conv1.weight):
            # bn0 + ReLU folded into conv1 (identity shortcut: the sum itself, through the alias output)
            y, part, s = bn_conv1x1(x.t, x.part, self.bn0, self.conv1.weight)
            h = self.bn1.forward_tiles(y, part)[0]
            pre = None
        elif isinstance(x, Fused):
            pre, s = self.bn0.forward_tiles(x.t, x.part)
        elif isinstance(x, tuple):
            pre, s = self.bn0.forward_add(*x)
        else:
            pre, s = self.bn0(x), x
        if self.shortcut is None:
            sc = s
        elif FUSED_1X1 and _fused_ok(self.conv1, pre) and self.shortcut.bias is None \
                and proj_pair_eligible(pre, self.shortcut.weight, self.shortcut.stride[0], self.conv1.weight):
            # projection shortcut + conv1 as one node: the two input gradients are summed inside conv1's dX GEMM, which
            # also reduces bn0's backward sums (pre feeds only this pair)
            sc, y, part = proj_pair(pre, self.shortcut.weight, self.shortcut.stride[0], self.conv1.weight,
                                    bn_input=True)
            h = self.bn1.forward_tiles(y, part)[0]
        elif _fused_ok(self.shortcut, pre):
            sc = conv1x1(pre, self.shortcut.weight)[0]
        else:
            sc = self.shortcut(pre)
        if h is not None:
            pass
        elif _fused_ok(self.conv1, pre):
            # pre feeds only conv1 when the shortcut is the identity (the shortcut then takes bn0's alias output s)
            y, part = conv1x1(pre, self.conv1.weight, stats=True, bn_input=self.shortcut is None)
            h = self.bn1.forward_tiles(y, part)[0]
        else:
            h = self.bn1(self.conv1(pre))
        if _fused3_ok(self.conv2, h):
            # 3x3 on the implicit-GEMM kernel: BN2's statistics in its epilogue; h (BN1's output) feeds only conv2
            y, part = conv3x3(h, self.conv2.weight, self.conv2.stride[0], stats=True, bn_input=True)
            if sc.shape[1] == self.conv3.out_channels and bn_conv_eligible(y, part, self.bn2, self.conv3.weight):
                # bn2 + ReLU folded into conv3 (+ the shortcut, BN statistics of the sum)
                return Fused(*bn_conv1x1(y, part, self.bn2, self.conv3.weight, residual=sc)[:2])
            h = self.bn2.forward_tiles(y, part)[0]
        else:
            h = self.bn2(self.conv2(h))
        if _fused_ok(self.conv3, h) and sc.shape[1] == self.conv3.out_channels:
            return Fused(*conv1x1(h, self.conv3.weight, residual=sc, stats=True, bn_input=True))
        return self.conv3(h), sc


class ResNetV2(nn.Module):
    def __init__(self, layers=(3, 4, 6, 3), num_classes: int = 1001):
        super().__init__()
        self.stem = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        blocks, cin = [], 64
        for i, (n, w) in enumerate(zip(layers, (64, 128, 256, 512))):
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(PreActBottleneck(cin, w, stride))
                cin = w * 4
        self.blocks = nn.Sequential(*blocks)
        self.post_bn = BatchNormReLU2d(cin)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):  # x: [B, 3, H, W] in [0, 1] (NHWC memory format preferred)
        # the stem on the hand-written MFMA kernel where eligible (bf16 channels_last 3-channel input, csrc/stem_conv.hip);
        # max-pool on the HIP NHWC kernels (1-byte argmax) on the GPU, F.max_pool2d elsewhere
        y = max_pool3s2(stem_conv(x, self.stem.weight) if stem_eligible(x, self.stem.weight) else self.stem(x))
        out = self.blocks(y)
        y, _ = self.post_bn.forward_tiles(out.t, out.part) if isinstance(out, Fused) else self.post_bn.forward_add(*out)
        # global average pool whose backward writes the channels_last gradient directly (a plain mean's / adaptive
        # pool's backward materialises a strided gradient that the final BN backward copied back to NHWC: ~85 us)
        return self.fc(global_avg_pool(y))


def resnet50_v2(num_classes: int = 1001) -> ResNetV2:
    return ResNetV2((3, 4, 6, 3), num_classes)


PREPROCESS_SCRIPT = """
def pre_process(img):
    # uint8 HWC image -> float NCHW in [0, 1]
    return img.float().div(255.0).permute(2, 0, 1).unsqueeze(0)

def post_process(logits):
    # TF-Hub class 0 is 'background': label = argmax - 1
    return logits.argmax(1) - 1
"""
