"""Direct RCCL all-reduce on the compute stream through torch's own communicator (csrc/rccl_direct.cpp).

torch.distributed over RCCL ("nccl" backend) runs each collective through ProcessGroupNCCL: a separate
stream, events both ways and work bookkeeping. For the W&D data-parallel step (one flat 82 KB gradient
bucket per step) that wrapper dominates; this module enqueues ncclAllReduce on the CURRENT stream with the
communicator torch already created (ProcessGroupNCCL._comm_ptr()), so the step is kernel -> all-reduce ->
kernel in stream order. Eager (not captured into a graph), so its failure modes are those of any eager RCCL
call."""
from __future__ import annotations

import ctypes
import functools
import os

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops._lib import I32, VP, sig


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("rccl_direct")
    f = {
        "load": sig(lib, "mifx_rccl_load", [ctypes.c_char_p]),
        "err": sig(lib, "mifx_rccl_last_error", [], ctypes.c_char_p),
        "allreduce": sig(lib, "mifx_rccl_allreduce_sum", [VP, VP, ctypes.c_size_t, I32, VP]),
    }
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    if f["load"](path.encode()) != 0:
        raise RuntimeError(f"RCCL load failed: {f['err']().decode()}")
    return f


def comm_ptr(pg=None, device: torch.device | None = None) -> int:
    """The ncclComm_t of pg's RCCL backend for `device` (forces its lazy initialisation first)."""
    pg = pg if pg is not None else dist.group.WORLD
    device = device or torch.device("cuda", torch.cuda.current_device())
    if dist.get_backend(pg) != "nccl":
        raise RuntimeError("direct RCCL needs the nccl (RCCL) backend")
    t = torch.zeros(1, device=device)
    dist.all_reduce(t, group=pg)  # materialise the communicator
    torch.cuda.synchronize(device)
    be = pg._get_backend(device)
    ptr = int(be._comm_ptr())
    if not ptr:
        raise RuntimeError("ProcessGroupNCCL returned a null communicator")
    return ptr


class DirectAllReduce:
    """In-place SUM all-reduce of a fixed fp32/bf16 CUDA buffer on the current stream. The arguments are
    prepared once so a call costs one ctypes call (a few us of host time)."""

    def __init__(self, buf: torch.Tensor, pg=None):
        if not buf.is_cuda or not buf.is_contiguous() or buf.dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("buffer must be a contiguous fp32/bf16 CUDA tensor")
        self.buf = buf
        self.comm = ctypes.c_void_p(comm_ptr(pg, buf.device))
        self._args = (self.comm, ctypes.c_void_p(buf.data_ptr()), ctypes.c_size_t(buf.numel()),
                      int(buf.dtype == torch.bfloat16))
        self._fn = _fns()["allreduce"]

    def __call__(self, stream: torch.cuda.Stream | None = None) -> None:
        s = stream or torch.cuda.current_stream(self.buf.device)
        rc = self._fn(*self._args, ctypes.c_void_p(s.cuda_stream))
        if rc != 0:
            raise RuntimeError(f"direct RCCL all-reduce failed ({rc}): {_fns()['err']().decode()}")
