"""Flat mixed-precision AdamW (csrc/adamw.hip): bf16 weights/grads in flat buffers, fp32 master +
moments, one launch per step, device-side step counter (graph-capturable). CPU reference included."""
from __future__ import annotations

import functools

import torch

from . import _lib
from ._lib import F32, I32, I64, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fn():
    lib = _lib.load("adamw")
    return sig(lib, "mifx_adamw_flat", [VP, VP, VP, VP, VP, I64, VP, F32, F32, F32, F32, F32, F32, VP])


@functools.lru_cache(maxsize=None)
def _fns_chunks():
    lib = _lib.load("adamw")
    return {"chunk": sig(lib, "mifx_adamw_chunk_size", []),
            "run": sig(lib, "mifx_adamw_chunks", [VP, VP, VP, VP, VP, VP, I32, VP, VP, VP, VP, F32, F32, F32, F32,
                                                  F32, F32, VP]),
            "run_noadv": sig(lib, "mifx_adamw_chunks_noadv", [VP, VP, VP, VP, VP, VP, I32, VP, VP, VP, VP, F32, F32,
                                                              F32, F32, F32, F32, VP]),
            "advance": sig(lib, "mifx_adamw_advance", [VP, VP])}


def chunk_size() -> int:
    return int(_fns_chunks()["chunk"]())


def adamw_chunks_(param: torch.Tensor, gptr: torch.Tensor, poff: torch.Tensor, bp: torch.Tensor, bo: torch.Tensor,
                  bn: torch.Tensor, master: torch.Tensor, m: torch.Tensor, v: torch.Tensor, step: torch.Tensor,
                  lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 0.0,
                  grad_scale: float = 1.0, advance: bool = True) -> None:
    """AdamW over flat bf16 weights / fp32 master+moments with each parameter's gradient read from its own
    tensor: gptr [P] uint64 device addresses (0 = no grad), poff [P] int64 flat offsets (multiples of 8),
    bp/bo/bn [nblocks] int32 chunk -> (parameter, element offset, length). See FlatAdamW. advance=False leaves the
    step counter (adamw_advance_ once after all launches of a split step)."""
    assert param.dtype == torch.bfloat16 and master.dtype == m.dtype == v.dtype == torch.float32
    assert gptr.dtype == torch.int64 and poff.dtype == torch.int64 and step.dtype == torch.int32
    assert bp.dtype == bo.dtype == bn.dtype == torch.int32 and bp.numel() == bo.numel() == bn.numel()
    check(_fns_chunks()["run" if advance else "run_noadv"](ptr(param), ptr(gptr), ptr(poff), ptr(bp), ptr(bo), ptr(bn), int(bp.numel()),
                               ptr(master), ptr(m), ptr(v), ptr(step), float(lr), float(beta1), float(beta2),
                               float(eps), float(weight_decay), float(grad_scale), stream_handle(param.device)),
          "mifx_adamw_chunks")


def adamw_flat_(param: torch.Tensor, grad: torch.Tensor, master: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                step: torch.Tensor, lr: float, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
                weight_decay: float = 0.0, grad_scale: float = 1.0) -> None:
    """In-place AdamW over flat 1-D buffers; `step` is an int32 device scalar advanced by one."""
    n = param.numel()
    if param.is_cuda:
        assert param.dtype == grad.dtype == torch.bfloat16 and master.dtype == m.dtype == v.dtype == torch.float32
        assert step.dtype == torch.int32 and all(t.numel() == n for t in (grad, master, m, v))
        check(_fn()(ptr(param), ptr(grad), ptr(master), ptr(m), ptr(v), n, ptr(step), float(lr), float(beta1),
                    float(beta2), float(eps), float(weight_decay), float(grad_scale), stream_handle(param.device)),
              "mifx_adamw_flat")
        return
    t = int(step.item()) + 1
    g = grad.float() * grad_scale
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1, bc2 = 1 - beta1 ** t, 1 - beta2 ** t
    master.mul_(1 - lr * weight_decay).addcdiv_(m, v.sqrt() / bc2 ** 0.5 + eps, value=-lr / bc1)
    param.copy_(master.to(param.dtype))
    step.add_(1)


def adamw_advance_(step: torch.Tensor) -> None:
    check(_fns_chunks()["advance"](ptr(step), stream_handle(step.device)), "mifx_adamw_advance")
