"""TF-semantics optimizers for the PyTorch reference path.

The canned DNNLinearCombinedClassifier (`taxi_utils.py:186-191`) trains its DNN with Adagrad
(lr 0.05, initial accumulator 0.1) and its linear part with FTRL (lr = min(0.2, 1/sqrt(#cols)),
lr_power -0.5, initial accumulator 0.1). These match TF's ApplyAdagrad / ApplyFtrl update rules
exactly (no epsilon), as does the fused HIP optimizer in csrc/wide_deep.hip.
"""
from __future__ import annotations

import functools
import os

import torch


class TFAdagrad(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 0.05, initial_accumulator_value: float = 0.1):
        super().__init__(params, dict(lr=lr, init=initial_accumulator_value))

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "acc" not in st:
                    st["acc"] = torch.full_like(p, g["init"])
                st["acc"].addcmul_(p.grad, p.grad)
                p.addcdiv_(p.grad, st["acc"].sqrt(), value=-g["lr"])


class Ftrl(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 0.2, lr_power: float = -0.5, initial_accumulator_value: float = 0.1,
                 l1: float = 0.0, l2: float = 0.0):
        super().__init__(params, dict(lr=lr, lr_power=lr_power, init=initial_accumulator_value, l1=l1, l2=l2))

    @torch.no_grad()
    def step(self, closure=None):
        for g in self.param_groups:
            lr, pw, l1, l2 = g["lr"], g["lr_power"], g["l1"], g["l2"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "acc" not in st:
                    st["acc"] = torch.full_like(p, g["init"])
                    st["lin"] = torch.zeros_like(p)
                acc, lin, grad = st["acc"], st["lin"], p.grad
                new_acc = acc + grad * grad
                if pw == -0.5:
                    sq_new, sq_old = new_acc.sqrt(), acc.sqrt()
                else:
                    sq_new, sq_old = new_acc.pow(-pw), acc.pow(-pw)
                lin.add_(grad - (sq_new - sq_old) / lr * p)
                quad = sq_new / lr + 2 * l2
                p.copy_(torch.where(lin.abs() > l1, (torch.sign(lin) * l1 - lin) / quad, torch.zeros_like(p)))
                acc.copy_(new_acc)


def make_optimizer(kind: str, params, lr: float, **kw) -> torch.optim.Optimizer:
    kind = kind.lower()
    if kind == "adagrad":
        return TFAdagrad(params, lr=lr, **kw)
    if kind == "ftrl":
        return Ftrl(params, lr=lr, **kw)
    if kind == "adam":
        return torch.optim.Adam(params, lr=lr, **kw)
    if kind == "sgd":
        return torch.optim.SGD(params, lr=lr, **kw)
    raise ValueError(f"unknown optimizer {kind}")


class FlatAdamW:
    """AdamW over a model whose parameters are re-homed as bf16 views of ONE flat buffer, with fp32 master
    weights / moments kept here. `step()` is a single fused HIP launch (mifx.ops.adamw).

    Gradients (`grads=`):
      * "own" (default on the GPU): autograd's own per-parameter gradient tensors are read in place by the
        chunked kernel (a per-step table of their addresses), `zero_grad()` sets them to None -- no zero-fill
        and no `grad += new` accumulate kernel per parameter per step;
      * "views": gradients are views of one flat gradient buffer that autograd accumulates into (one memset
        per `zero_grad()`); the flat kernel is then hipGraph-capturable (device-side step counter)."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 dtype: torch.dtype = torch.bfloat16, grads: str | None = None, overlap: bool | None = None,
                 bucket_elems: int = 8 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.lr, self.betas, self.eps, self.wd = lr, betas, eps, weight_decay
        dev = self.params[0].device
        if grads is None:
            grads = "own" if dev.type == "cuda" and dtype == torch.bfloat16 else "views"
        if grads not in ("own", "views"):
            raise ValueError("grads must be 'own' or 'views'")
        if grads == "own" and (dev.type != "cuda" or dtype != torch.bfloat16):
            raise ValueError("grads='own' needs bf16 parameters on the GPU")
        self.mode = grads
        align = 8 if grads == "own" else 1  # 16-byte aligned bf16 / 32-byte fp32 vectors per parameter
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += (p.numel() + align - 1) // align * align
        n = off
        self.n = n
        self.flat = torch.zeros(n, device=dev, dtype=dtype)
        self.flat_grad = torch.zeros(n, device=dev, dtype=dtype) if grads == "views" else None
        self.master = torch.zeros(n, device=dev, dtype=torch.float32)
        self.m = torch.zeros(n, device=dev, dtype=torch.float32)
        self.v = torch.zeros(n, device=dev, dtype=torch.float32)
        self.step_count = torch.zeros((), device=dev, dtype=torch.int32)
        with torch.no_grad():
            for p, off in zip(self.params, offs):
                k = p.numel()
                self.master[off:off + k].copy_(p.detach().reshape(-1).float())
                self.flat[off:off + k].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + k].view(p.shape)
                p.grad = self.flat_grad[off:off + k].view(p.shape) if grads == "views" else None
        if grads == "own":
            from ..ops.adamw import chunk_size

            ch = chunk_size()
            bp, bo, bn = [], [], []
            for i, p in enumerate(self.params):
                for o in range(0, p.numel(), ch):
                    bp.append(i)
                    bo.append(o)
                    bn.append(min(ch, p.numel() - o))
            self.poff = torch.tensor(offs, dtype=torch.int64, device=dev)
            self._gptr = torch.zeros(len(self.params), dtype=torch.int64, device=dev)  # grad addresses
            self._capture_host = torch.zeros(len(self.params), dtype=torch.int64).pin_memory()
            self._addr = None
            self.bp, self.bo, self.bn = (torch.tensor(x, dtype=torch.int32, device=dev) for x in (bp, bo, bn))
            # overlap (opt-in: overlap=True or MIFX_ADAMW_OVERLAP=1): in a CAPTURED step, the update of each bucket of
            # ~bucket_elems consecutive parameters is launched on a side stream as soon as autograd has accumulated
            # the last gradient of the bucket (post-accumulate-grad hooks), so the memory-bound update of layer L
            # runs under the compute-bound backward of layers < L; step() launches what is left, joins the side
            # stream and advances the step counter once. Every bucket reads the same step value, so the update is
            # the single-launch update, bucket by bucket (same kernel, same per-element math). Measured SLOWER in the
            # BERT-base step (7.18 vs 6.38 ms on MI355X, profiles/archive/bert_adamw_overlap_r3.txt): the bucket launches fill
            # every CU with memory-bound blocks beside the backward's one-workgroup-per-CU GEMMs, which lose more
            # than the ~0.5 ms update that is hidden.
            if overlap is None:
                overlap = os.environ.get("MIFX_ADAMW_OVERLAP", "0") == "1"
            self.overlap = bool(overlap)
            if self.overlap:
                self._buckets, cur, acc = [], [], 0
                for i, p in enumerate(self.params):
                    cur.append(i)
                    acc += p.numel()
                    if acc >= bucket_elems:
                        self._buckets.append(cur)
                        cur, acc = [], 0
                if cur:
                    self._buckets.append(cur)
                self._bucket_of = {i: b for b, idx in enumerate(self._buckets) for i in idx}
                self._bchunks = []
                for idx in self._buckets:
                    sel = [k for k, pi in enumerate(bp) if idx[0] <= pi <= idx[-1]]
                    self._bchunks.append(tuple(torch.tensor([x[k] for k in sel], dtype=torch.int32, device=dev)
                                               for x in (bp, bo, bn)))
                self._ov_host = torch.zeros(len(self.params), dtype=torch.int64).pin_memory()
                self._ov_side = torch.cuda.Stream(dev)
                self._ov_ready = [0] * len(self._buckets)
                self._ov_launched = [False] * len(self._buckets)
                self._ov_active = False
                self._ov_captured = False
                for i, p in enumerate(self.params):
                    p.register_post_accumulate_grad_hook(functools.partial(self._on_grad, i))

    @torch.no_grad()
    def reload_master(self) -> None:
        """Re-derive the fp32 master weights from the bf16 parameters after they were written from outside the
        optimizer (load_state_dict into the flat views, a warm start): otherwise the next step would overwrite the
        loaded weights with the stale master copy."""
        self.master.copy_(self.flat.float())

    # ---------------------------------------------------------------- overlapped update (captured steps)
    def _on_grad(self, i: int, p: torch.Tensor) -> None:
        if not (self._ov_active and torch.cuda.is_current_stream_capturing()):
            return
        b = self._bucket_of[i]
        self._ov_ready[b] += 1
        if self._ov_ready[b] == len(self._buckets[b]) and not self._ov_launched[b]:
            self._launch_bucket(b)

    def _launch_bucket(self, b: int) -> None:
        from ..ops.adamw import adamw_chunks_

        idx = self._buckets[b]
        i0, i1 = idx[0], idx[-1] + 1
        host = self._ov_host.numpy()
        for i in idx:
            g = self.params[i].grad
            if g is not None and (g.dtype != torch.bfloat16 or not g.is_contiguous() or g.device != self.flat.device):
                raise RuntimeError("FlatAdamW(grads='own') needs contiguous bf16 gradients on the parameter's device")
            host[i] = 0 if g is None else g.data_ptr()
        cur = torch.cuda.current_stream(self.flat.device)
        self._ov_side.wait_stream(cur)  # the bucket's gradients (and the backward kernels that read its weights)
        with torch.cuda.stream(self._ov_side):
            # captured H2D copy: reads the pinned table on every replay (the captured gradients keep their
            # addresses, so the table is written once, here)
            self._gptr[i0:i1].copy_(self._ov_host[i0:i1], non_blocking=True)
            bpb, bob, bnb = self._bchunks[b]
            adamw_chunks_(self.flat, self._gptr, self.poff, bpb, bob, bnb, self.master, self.m, self.v,
                          self.step_count, self.lr, self.betas[0], self.betas[1], self.eps, self.wd, advance=False)
        self._ov_launched[b] = True

    def begin_capture(self) -> None:
        """Arm the overlapped update for the step about to be captured (one captured step per optimizer)."""
        if self.mode == "own" and self.overlap:
            if self._ov_captured:
                raise RuntimeError("FlatAdamW overlap: one captured step per optimizer")
            self._ov_ready = [0] * len(self._buckets)
            self._ov_launched = [False] * len(self._buckets)
            self._ov_active = True

    def zero_grad(self, set_to_none: bool = True) -> None:
        if self.mode == "own":
            for p in self.params:
                p.grad = None
        else:  # grads stay views of the flat buffer
            self.flat_grad.zero_()

    def step(self) -> None:
        from ..ops.adamw import adamw_chunks_, adamw_flat_

        if self.mode == "views":
            adamw_flat_(self.flat, self.flat_grad, self.master, self.m, self.v, self.step_count, self.lr,
                        self.betas[0], self.betas[1], self.eps, self.wd)
            return
        addr = []
        for p in self.params:
            g = p.grad
            if g is not None and (g.dtype != torch.bfloat16 or not g.is_contiguous() or g.device != p.device):
                raise RuntimeError("FlatAdamW(grads='own') needs contiguous bf16 gradients on the parameter's device")
            addr.append(0 if g is None else g.data_ptr())
        addr = tuple(addr)
        if self.overlap and self._ov_active and torch.cuda.is_current_stream_capturing():
            from ..ops.adamw import adamw_advance_

            for b in range(len(self._buckets)):  # buckets whose last gradient never arrived (unused parameters)
                if not self._ov_launched[b]:
                    self._launch_bucket(b)
            torch.cuda.current_stream(self.flat.device).wait_stream(self._ov_side)
            adamw_advance_(self.step_count)
            self._ov_active, self._ov_captured = False, True
            self._capture_host = None
            return
        if torch.cuda.is_current_stream_capturing():
            # hipGraph capture: no pinned allocation is allowed here, so the table goes through the pinned
            # buffer reserved at construction; the captured copy reads it on every replay, so it is never
            # written again (the captured gradients keep their addresses on every replay)
            if self._capture_host is None:
                raise RuntimeError("FlatAdamW(grads='own') supports one captured step per optimizer")
            self._capture_host.numpy()[:] = addr
            self._gptr.copy_(self._capture_host, non_blocking=True)
            self._capture_host, self._addr = None, addr
        elif addr != self._addr:  # eager: upload only when autograd handed out new gradient addresses
            self._gptr.copy_(torch.tensor(addr, dtype=torch.int64).pin_memory(), non_blocking=True)
            self._addr = addr
        adamw_chunks_(self.flat, self._gptr, self.poff, self.bp, self.bo, self.bn, self.master, self.m, self.v,
                      self.step_count, self.lr, self.betas[0], self.betas[1], self.eps, self.wd)

    def state_dict(self) -> dict:
        return {"master": self.master, "m": self.m, "v": self.v, "step": self.step_count}
