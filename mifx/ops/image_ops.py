"""Fused crop + flip + normalize for HBM-resident uint8 image datasets (csrc/image_ops.hip).

The host reference reproduces the device Philox stream bit-exactly (mifx.ops.dp.philox4x32), so
CPU and GPU augmentations pick the same crops and flips."""
from __future__ import annotations

import ctypes
import functools

import numpy as np
import torch

from . import _lib
from ._lib import I32, VP, check, ptr, sig, stream_handle

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("image_ops")
    return {"cfn": sig(lib, "mifx_img_crop_flip_norm", [VP, VP, I32, I32, I32, I32, I32, I32, I32, ctypes.c_ulonglong,
                                                         ctypes.c_uint, VP, VP, I32, VP, VP])}


def crop_params(B: int, Hin: int, Win: int, Hout: int, Wout: int, train: bool, seed: int, step: int):
    if not train:
        z = np.zeros(B, np.int64)
        return z + (Hin - Hout) // 2, z + (Win - Wout) // 2, z
    from .dp import philox4x32

    x, y, zz, _ = philox4x32(np.arange(B, dtype=np.uint32), step & 0xFFFFFFFF, 0x1234, 0, seed)
    return (x % np.uint32(Hin - Hout + 1)).astype(np.int64), (y % np.uint32(Win - Wout + 1)).astype(np.int64), \
        (zz & np.uint32(1)).astype(np.int64)


def crop_flip_normalize(images: torch.Tensor, idx: torch.Tensor, out_hw=(224, 224), train: bool = True,
                        seed: int = 0, step: int = 0, mean=IMAGENET_MEAN, std=IMAGENET_STD,
                        dtype=torch.bfloat16) -> torch.Tensor:
    """images uint8 [N, H, W, C]; idx [B] -> [B, C, Hout, Wout] in channels_last memory format."""
    N, Hin, Win, C = images.shape
    Hout, Wout = out_hw
    B = int(idx.numel())
    if images.is_cuda:
        out = torch.empty(B, Hout, Wout, C, device=images.device, dtype=dtype)
        m = torch.tensor(mean, device=images.device, dtype=torch.float32)
        inv = 1.0 / torch.tensor(std, device=images.device, dtype=torch.float32)
        idx32 = idx.to(device=images.device, dtype=torch.int32).contiguous()
        check(_fns()["cfn"](ptr(images), ptr(idx32), B, Hin, Win, C, Hout, Wout, int(train), seed, step, ptr(m),
                            ptr(inv), 1 if dtype == torch.bfloat16 else 0, ptr(out), stream_handle(images.device)),
              "mifx_img_crop_flip_norm")
        return out.permute(0, 3, 1, 2)  # NCHW view with channels_last strides
    oy, ox, flip = crop_params(B, Hin, Win, Hout, Wout, train, seed, step)
    outs = []
    for b in range(B):
        im = images[int(idx[b]), oy[b]:oy[b] + Hout, ox[b]:ox[b] + Wout].float() / 255.0
        if flip[b]:
            im = im.flip(1)
        outs.append(im)
    x = (torch.stack(outs) - torch.tensor(mean)) / torch.tensor(std)
    return x.to(dtype).permute(0, 3, 1, 2)
