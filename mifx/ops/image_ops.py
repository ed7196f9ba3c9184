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
                                                         ctypes.c_uint, VP, VP, VP, I32, VP, VP])}


@functools.lru_cache(maxsize=64)
def _norm_consts(device: str, mean: tuple, std: tuple):
    """Device mean / 1/std (cached: no host-to-device copy per call, so the call can be captured in a hipGraph)."""
    m = torch.tensor(mean, device=device, dtype=torch.float32)
    return m, 1.0 / torch.tensor(std, device=device, dtype=torch.float32)


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
                        dtype=torch.bfloat16, step_dev: torch.Tensor | None = None) -> torch.Tensor:
    """images uint8 [N, H, W, C]; idx [B] -> [B, C, Hout, Wout] in channels_last memory format. step_dev (GPU): a
    device int64 [1] step counter the kernel reads instead of `step` (for steps captured into a hipGraph)."""
    N, Hin, Win, C = images.shape
    Hout, Wout = out_hw
    B = int(idx.numel())
    if images.is_cuda:
        out = torch.empty(B, Hout, Wout, C, device=images.device, dtype=dtype)
        m, inv = _norm_consts(str(images.device), tuple(float(v) for v in mean), tuple(float(v) for v in std))
        idx32 = idx.to(device=images.device, dtype=torch.int32).contiguous()
        if step_dev is not None and (step_dev.dtype != torch.int64 or step_dev.device != images.device):
            raise ValueError("step_dev must be an int64 tensor on the images' device")
        check(_fns()["cfn"](ptr(images), ptr(idx32), B, Hin, Win, C, Hout, Wout, int(train), seed, step,
                            ptr(step_dev), ptr(m),
                            ptr(inv), 1 if dtype == torch.bfloat16 else 0, ptr(out), stream_handle(images.device)),
              "mifx_img_crop_flip_norm")
        return out.permute(0, 3, 1, 2)  # NCHW view with channels_last strides
    if step_dev is not None:
        step = int(step_dev.reshape(-1)[0])
    oy, ox, flip = crop_params(B, Hin, Win, Hout, Wout, train, seed, step)
    outs = []
    for b in range(B):
        im = images[int(idx[b]), oy[b]:oy[b] + Hout, ox[b]:ox[b] + Wout].float() / 255.0
        if flip[b]:
            im = im.flip(1)
        outs.append(im)
    x = (torch.stack(outs) - torch.tensor(mean)) / torch.tensor(std)
    return x.to(dtype).permute(0, 3, 1, 2)
