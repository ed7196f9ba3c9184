"""ResNet-50 v2 (pre-activation) image classifier, 1001 classes (TF-Hub `resnet_v2_50` layout used by
the RedisAI demo, `notebooks/redis/utils/model_saver.py:1-14`; KN17). Channels-last so MIOpen runs
its NHWC MFMA convolutions; `inference_mode` + bf16 autocast for serving."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.bn_relu import BatchNormReLU2d
from ..ops.pool import max_pool3s2


class PreActBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int):
        super().__init__()
        cout = width * self.expansion
        self.bn0 = BatchNormReLU2d(cin)  # every BN of the pre-activation net feeds a ReLU: fused
        self.shortcut = nn.Conv2d(cin, cout, 1, stride=stride, bias=False) if (stride != 1 or cin != cout) else None
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = BatchNormReLU2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNormReLU2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)

    def forward(self, x):
        """x: a tensor, or the (branch, shortcut) pair of the previous block whose sum is this block's
        input -- the residual add then happens inside bn0's fused kernels (fwd and bwd). Returns the
        un-added (branch, shortcut) pair for the next block / the final BN."""
        if isinstance(x, tuple):
            pre, s = self.bn0.forward_add(*x)
        else:
            pre, s = self.bn0(x), x
        sc = self.shortcut(pre) if self.shortcut is not None else s
        y = self.conv1(pre)
        y = self.conv2(self.bn1(y))
        y = self.conv3(self.bn2(y))
        return y, sc


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
        y = max_pool3s2(self.stem(x))  # HIP NHWC kernels (1-byte argmax) on the GPU, F.max_pool2d elsewhere
        y, _ = self.post_bn.forward_add(*self.blocks(y))
        # global average pool whose backward keeps the channels_last layout (a plain mean's backward
        # materialises an NCHW gradient, copied back to NHWC by the final BN backward)
        return self.fc(F.adaptive_avg_pool2d(y, 1).flatten(1))


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
