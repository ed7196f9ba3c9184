"""Image CNN families from the reference notebooks / research code (PyTorch, channels-last NHWC
so MIOpen picks its NHWC implicit-GEMM (MFMA) convolution kernels on gfx950).

* `MnistDPCNN` — DP-SGD tutorial CNN (`privacy/tutorials/mnist_dpsgd_tutorial.py:42-58`):
  Conv16 8x8 s2 SAME -> MaxPool2 s1 -> Conv32 4x4 s2 VALID -> MaxPool2 s1 -> Dense32 -> Dense10.
* `PateCNN` — PATE-2017 `deep_cnn.inference` (`research/pate_2017/deep_cnn.py:84-191`):
  conv5x5->64, maxpool3 s2, LRN(4, 1, 0.001/9, 0.75), conv5x5->128, LRN, maxpool3 s2, fc384, fc192, fc C;
  `deeper=True` gives `inference_deeper` (3x3 convs 96/96/96s2/192/192/192s2/192, fc192, fc C).
* `FashionCNN` — serving notebook model (`serving/Predict_Fashion_MNIST.ipynb`): Conv8 3x3 s2 + Dense10.
* `TpuMnistCNN` — TPU notebook model (`tpu/Keras_MNIST_TPU.ipynb`): Conv32-Pool-Conv64-Pool-Conv64-
  Dense64-Dropout-Dense10.
TF "SAME" padding is reproduced exactly (asymmetric when needed) so shapes match the reference. With
MIFX_SMALL_CONV=1 the few-channel first layers run on the direct fp32 HIP kernels (csrc/conv_small.hip; opt-in:
MIOpen measured faster, mifx/ops/conv_small.py); the PATE ensembles use the grouped MFMA kernel (csrc/gconv.hip)."""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import cnn_ops, pool
from ..ops.conv_small import SmallConv2d


def _same_pad(x: torch.Tensor, k: int, s: int, value: float = 0.0) -> torch.Tensor:
    """TF SAME padding for NCHW tensors (pads more on the bottom/right when odd)."""
    h, w = x.shape[-2:]
    ph = max((math.ceil(h / s) - 1) * s + k - h, 0)
    pw = max((math.ceil(w / s) - 1) * s + k - w, 0)
    if ph == 0 and pw == 0:
        return x
    return F.pad(x, (pw // 2, pw - pw // 2, ph // 2, ph - ph // 2), value=value)


class SameConv2d(SmallConv2d):
    """TF "SAME" conv (few-channel layers on the direct HIP kernels when MIFX_SMALL_CONV=1, else nn.Conv2d)."""

    def __init__(self, cin, cout, k, stride=1):
        super().__init__(cin, cout, k, stride=stride, same=True)


def same_maxpool(x, k, s):
    if k == 3 and s == 2:  # NHWC bf16 on the GPU: HIP kernels (csrc/pool.hip), 1-byte argmax
        y = pool.max_pool3s2_same(x)
        if y is not None:
            return y
    return F.max_pool2d(_same_pad(x, k, s, value=-math.inf), k, s)


def _he_normal_(m: nn.Module) -> None:
    for mod in m.modules():
        if isinstance(mod, (nn.Conv2d, nn.Linear)):
            nn.init.kaiming_normal_(mod.weight, nonlinearity="relu")
            nn.init.zeros_(mod.bias)


class MnistDPCNN(nn.Module):
    def __init__(self, num_classes: int = 10):
        super().__init__()
        self.conv1 = SameConv2d(1, 16, 8, stride=2)
        self.conv2 = SmallConv2d(16, 32, 4, stride=2)
        self.fc1 = nn.Linear(32 * 4 * 4, 32)
        self.fc2 = nn.Linear(32, num_classes)
        _he_normal_(self)

    def forward(self, x):  # x: [B, 28, 28] or [B, 1, 28, 28]
        if x.dim() == 3:
            x = x.unsqueeze(1)
        y = F.max_pool2d(self.conv1(x), 2, 1)   # 14x14 -> 13x13
        y = F.max_pool2d(self.conv2(y), 2, 1)   # 5x5 -> 4x4
        y = self.fc1(y.flatten(1))               # tutorial uses linear Dense(32)
        return self.fc2(y)


class PateCNN(nn.Module):
    def __init__(self, in_ch: int = 1, num_classes: int = 10, image: int = 28, deeper: bool = False,
                 dropout: bool = False):
        super().__init__()
        self.deeper, self.dropout = deeper, dropout
        if not deeper:
            self.c1 = SameConv2d(in_ch, 64, 5)
            self.c2 = SameConv2d(64, 128, 5)
            s = math.ceil(math.ceil(image / 2) / 2)
            self.f3 = nn.Linear(128 * s * s, 384)
            self.f4 = nn.Linear(384, 192)
            self.out = nn.Linear(192, num_classes)
        else:
            chans = [(in_ch, 96, 1), (96, 96, 1), (96, 96, 2), (96, 192, 1), (192, 192, 1), (192, 192, 2),
                     (192, 192, 1)]
            self.convs = nn.ModuleList([SameConv2d(a, b, 3, st) for a, b, st in chans])
            s = math.ceil(math.ceil(image / 2) / 2)
            self.f1 = nn.Linear(192 * s * s, 192)
            self.out = nn.Linear(192, num_classes)
        for mod in self.modules():
            if isinstance(mod, (nn.Conv2d, nn.Linear)):
                nn.init.trunc_normal_(mod.weight, std=0.05 if isinstance(mod, nn.Conv2d) else 0.04)
                nn.init.constant_(mod.bias, 0.1 if isinstance(mod, nn.Linear) else 0.0)

    @staticmethod
    def _lrn(x):  # tf.nn.lrn(depth_radius=4, bias=1.0, alpha=0.001/9, beta=0.75)
        # NHWC GPU activations: HIP LRN fwd/bwd kernels (csrc/cnn_ops.hip); else torch's LRN
        return cnn_ops.lrn(x, depth_radius=4, bias=1.0, alpha=0.001 / 9.0, beta=0.75)

    def forward(self, x):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        drop = self.dropout and self.training
        if not self.deeper:
            y = F.relu(self.c1(x))
            y = F.dropout(y, 0.7, drop)  # tf keep_prob 0.3
            y = self._lrn(same_maxpool(y, 3, 2))
            y = F.relu(self.c2(y))
            y = F.dropout(y, 0.7, drop)
            y = same_maxpool(self._lrn(y), 3, 2)
            y = F.dropout(F.relu(self.f3(y.flatten(1))), 0.5, drop)
            y = F.dropout(F.relu(self.f4(y)), 0.5, drop)
            return self.out(y)
        y = x
        for i, c in enumerate(self.convs):
            y = F.relu(c(y))
            if i in (2, 5):
                y = F.dropout(y, 0.5, drop)
        y = F.dropout(F.relu(self.f1(y.flatten(1))), 0.5, drop)
        return self.out(y)


class FashionCNN(nn.Module):
    """`Predict_Fashion_MNIST.ipynb` cell 8: Conv2D(8, 3x3, stride 2, relu) -> Dense(10, softmax).
    `forward` returns class probabilities (what the served model answers); train on `logits`."""

    def __init__(self, num_classes: int = 10):
        super().__init__()
        # the direct HIP conv by default here: the whole Fashion training step measured 0.43 vs 0.54 ms/step on
        # MIOpen (profiles/archive/cnn_small_conv_r3.jsonl; MIFX_SMALL_CONV=0 forces the library)
        self.conv = SmallConv2d(1, 8, 3, stride=2, prefer=True)
        self.fc = nn.Linear(8 * 13 * 13, num_classes)

    def logits(self, x):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        return self.fc(F.relu(self.conv(x)).flatten(1))

    def forward(self, x):
        return F.softmax(self.logits(x), dim=-1)


class TpuMnistCNN(nn.Module):
    def __init__(self, num_classes: int = 10, dropout: float = 0.5):
        super().__init__()
        self.c1 = SmallConv2d(1, 32, 3)
        self.c2 = SmallConv2d(32, 64, 3)
        self.c3 = SmallConv2d(64, 64, 3)
        self.fc = nn.Linear(64 * 3 * 3, 64)
        self.out = nn.Linear(64, num_classes)
        self.p = dropout

    def forward(self, x):
        if x.dim() == 3:
            x = x.unsqueeze(1)
        y = F.max_pool2d(F.relu(self.c1(x)), 2)
        y = F.max_pool2d(F.relu(self.c2(y)), 2)
        y = F.relu(self.c3(y))
        y = F.dropout(F.relu(self.fc(y.flatten(1))), self.p, self.training)
        return self.out(y)


def to_channels_last(model: nn.Module) -> nn.Module:
    """NHWC weights/activations: MIOpen's MFMA implicit-GEMM path on gfx950."""
    return model.to(memory_format=torch.channels_last)


class EMA:
    """Exponential moving average of weights (`deep_cnn.py:419-422`, decay 0.9999), applied in-place
    with fused multi-tensor ops after each optimizer step."""

    def __init__(self, model: nn.Module, decay: float = 0.9999):
        self.decay = decay
        self.shadow = [p.detach().clone() for p in model.parameters()]
        self.params = list(model.parameters())

    @torch.no_grad()
    def update(self) -> None:
        torch._foreach_lerp_(self.shadow, [p.detach() for p in self.params], 1.0 - self.decay)

    @torch.no_grad()
    def copy_to(self, model: nn.Module) -> None:
        for s, p in zip(self.shadow, model.parameters()):
            p.copy_(s)
