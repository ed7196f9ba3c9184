"""Multi-tensor fused SGD (csrc/sgd.hip): weight decay, momentum, dampening and Nesterov for a list of fp32
parameters in ONE launch, learning rate read from a device tensor (graph-capturable). `FusedSGDTables` builds the
per-tensor address / chunk tables once, outside any capture; `sgd_reference_` is the torch.optim.SGD foreach
update it replaces (the parity check of tests/test_sgd_fused.py)."""
from __future__ import annotations

import functools

import torch

from . import _lib
from ._lib import F32, I32, VP, check, ptr, sig, stream_handle


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("sgd")
    return {"chunk": sig(lib, "mifx_sgd_chunk_size", []),
            "run": sig(lib, "mifx_sgd_chunks", [VP, VP, VP, VP, VP, VP, VP, I32, VP, F32, F32, I32, VP])}


def _dense(t: torch.Tensor) -> bool:
    """Non-overlapping and dense: the strides, sorted, are the running products of the sizes (any dim order)."""
    expect = 1
    for st, sz in sorted((st, sz) for sz, st in zip(t.shape, t.stride()) if sz != 1):
        if st != expect:
            return False
        expect *= sz
    return True


class FusedSGDTables:
    """Device tables for one fused update of `params` (fp32, CUDA) with their momentum `bufs` and a per-tensor
    weight decay; the gradients' addresses are set per step (`set_grads`). The tables hold raw addresses: rebuild
    them (`matches`) when a parameter or momentum buffer is reallocated."""

    CAPTURES = 4  # graph captures one table set can serve (each keeps its own pinned address buffer)

    def __init__(self, params, bufs, wds, grads=None):
        dev = params[0].device
        # the update is elementwise, so any dense layout works (channels_last convolution weights) as long as a
        # parameter, its gradient and its momentum buffer share it: element i of one is element i of the others
        for t in (*params, *bufs):
            if t.dtype != torch.float32 or not t.is_cuda or not _dense(t):
                raise ValueError("fused SGD: dense fp32 CUDA tensors only")
        for p, b in zip(params, bufs):
            if not (p.shape == b.shape and p.stride() == b.stride()):
                raise ValueError("fused SGD: param / momentum layouts differ")
        ch = int(_fns()["chunk"]())
        tp, to, tn = [], [], []
        for i, p in enumerate(params):
            for o in range(0, p.numel(), ch):
                tp.append(i)
                to.append(o)
                tn.append(min(ch, p.numel() - o))
        self.params, self.bufs = list(params), list(bufs)  # the addresses stay valid while the tables live
        self.key = tuple(t.data_ptr() for t in (*params, *bufs))
        addr = lambda ts: torch.tensor([t.data_ptr() for t in ts], dtype=torch.int64, device=dev)  # noqa: E731
        self.pp, self.bp = addr(params), addr(bufs)
        self.gp = torch.zeros(len(params), dtype=torch.int64, device=dev)
        self._gp_host = torch.zeros(len(params), dtype=torch.int64).pin_memory()
        self.wd = torch.tensor([float(w) for w in wds], dtype=torch.float32, device=dev)
        self.tp, self.to, self.tn = (torch.tensor(x, dtype=torch.int32, device=dev) for x in (tp, to, tn))
        self.nblocks = len(tp)
        self.grads = None
        self._captured_hosts: list = []
        self._spare_hosts = [torch.zeros(len(params), dtype=torch.int64).pin_memory() for _ in range(self.CAPTURES)]
        if grads is not None:
            self.set_grads(grads)

    def matches(self, params, bufs) -> bool:
        return self.key == tuple(t.data_ptr() for t in (*params, *bufs))

    def grads_ok(self, grads) -> bool:
        return len(grads) == len(self.params) and all(
            g is not None and g.dtype == torch.float32 and g.shape == p.shape and g.stride() == p.stride()
            for g, p in zip(grads, self.params))

    def set_grads(self, grads) -> None:
        """Point the update at this step's gradient tensors: a pinned-host -> device copy of their addresses,
        so inside a capture it becomes a graph node (gradients produced in the graph's private pool keep their
        addresses on every replay)."""
        if not self.grads_ok(grads):
            raise ValueError("fused SGD: gradient layouts differ from their parameters'")
        capturing = torch.cuda.is_current_stream_capturing()
        if capturing:
            # the copy node re-reads its host buffer on every replay: give each capture a buffer of its own (pinned
            # ahead of time: no host allocation inside a capture), never written again, so a later set_grads cannot
            # retarget a captured graph
            if not self._spare_hosts:
                raise RuntimeError("fused SGD: more captures than reserved address buffers; rebuild the tables")
            host = self._spare_hosts.pop()
            self._captured_hosts.append(host)
        else:  # eager: the pinned buffer may still feed an earlier asynchronous copy
            torch.cuda.current_stream(self.gp.device).synchronize()
            host = self._gp_host
        for i, g in enumerate(grads):
            host[i] = g.data_ptr()
        self.gp.copy_(host, non_blocking=True)
        self.grads = list(grads)

    def step(self, neg_lr: torch.Tensor, momentum: float, dampening: float, nesterov: bool) -> None:
        """One update. The kernel writes the parameters through raw addresses, so their version counters are bumped
        here (at call / capture time): consumers keyed on w._version (mifx.ops.weight_prep bf16 images) then see
        the weights as changed instead of serving images from before the update."""
        if self.grads is None:
            raise RuntimeError("fused SGD: set_grads() before step()")
        check(_fns()["run"](ptr(self.pp), ptr(self.gp), ptr(self.bp), ptr(self.wd), ptr(self.tp), ptr(self.to),
                            ptr(self.tn), self.nblocks, ptr(neg_lr), float(momentum), float(dampening),
                            int(bool(nesterov)), stream_handle(neg_lr.device)), "mifx_sgd_chunks")
        torch.autograd.graph.increment_version(self.params)


@torch.no_grad()
def sgd_reference_(params, grads, bufs, wd: float, momentum: float, dampening: float, nesterov: bool,
                   neg_lr: torch.Tensor) -> None:
    """torch.optim.SGD's foreach update with the learning rate as a device tensor (-lr)."""
    if wd:
        grads = torch._foreach_add(grads, params, alpha=wd)
    torch._foreach_mul_(bufs, momentum)
    torch._foreach_add_(bufs, grads, alpha=1 - dampening)
    upd = torch._foreach_add(grads, bufs, alpha=momentum) if nesterov else [b.clone() for b in bufs]
    torch._foreach_mul_(upd, neg_lr)
    torch._foreach_add_(params, upd)
