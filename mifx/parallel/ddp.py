"""Bucketed data-parallel gradient synchronisation (one process per GPU, RCCL over xGMI).

Replaces the reference's delegated DP mechanisms — TFJob parameter servers, MPIJob/Horovod ring
all-reduce, PyTorchJob DDP (`tf-job-simple-v1beta2.jsonnet:22-74`,
`mpi-job.libsonnet:22-85`, `pytorch-job.jsonnet:63-81`) — with an in-process engine:

* gradients are packed into flat buckets in reverse registration order (≈ backward order), so the
  first bucket is complete while backward is still producing the rest;
* each bucket's all-reduce is launched the moment its last gradient is accumulated (post-accumulate
  hook) on a dedicated communication stream, overlapping RCCL with the remaining backward kernels;
* bucket size defaults to 32 MiB: on MI355X a ring all-reduce over point-to-point xGMI is per-link
  bandwidth bound (≈150 GB/s/link), so a bucket has to be several MB before the ring's
  2(N-1)/N·S/BW term dominates its ≈10-20 µs latency term, and few buckets keep the launch count low
  (the 288 GB HBM per GPU makes the flat buffers free);
* optional bf16 wire format halves xGMI bytes for bandwidth-bound models (fp32 accumulate on the
  receiving side is RCCL's; the master gradient stays fp32).

* buckets launch in bucket order on every rank (a bucket completing early waits for its predecessors), so the
  collective sequence is the same on all ranks whatever order autograd finished them in;
* with deferred weight gradients (grouped flushes, mifx.ops.gemm.deferred_weight_grads) the flushes of runs of complete
  buckets are coalesced (flush_min_wgs); by default ONE flush after the backward, then every bucket's exchange;
* exchange="ipc" replaces the RCCL collective by the peer-memory two-shot all-reduce of csrc/tp_allreduce.hip in fp32
  (publish / reduce-scatter / all-gather kernels synchronised by device-side epoch flags, rank-order sum scaled by
  1 / world in the kernel: identical bits on every rank): no host collective, so the whole data-parallel step --
  forward, backward with the bucket exchanges overlapped on the side stream, optimizer -- captures into ONE hipGraph
  (mifx.trainer.resnet_trainer). exchange="auto" takes it on CUDA when every rank can map its peers' memory (agreed
  over the group; RCCL otherwise).

`DataParallel.finish()` (or `step_ready()`) waits for outstanding work and writes averaged gradients
back into `param.grad`. With `grad_as_bucket_view=True` there is nothing to write back: every `param.grad` IS a
view of its bucket (same strides as the parameter, channels_last included), autograd accumulates straight into
the bucket, the all-reduce runs in place and the average is one scale per bucket -- no copy into or out of the
buckets (call `zero_grad()` instead of the optimizer's). Works unchanged on gloo/CPU, which is how the tests
exercise it."""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field

import torch
import torch.distributed as dist


# diagnostic: where the bucket exchange runs -- "side" (default: the communication stream, overlapping the backward),
# "main" (the compute stream), "join" (side stream, joined right after each launch), "copy" (no exchange: the bucket
# copied out and back in place on the side stream)
_COMM_DIAG = os.environ.get("MIFX_DP_COMM", "side")
# several buckets launched together fork the communication stream ONCE: one wait per bucket with no compute-stream
# work in between lost the ordering of the consecutive exchanges in captured graphs (they overlapped on the shared
# peer buffers; profiles/resnet_dp_flush_r6.md). MIFX_DP_FORK_ONCE=0 restores the old form (diagnostic).
_FORK_ONCE = os.environ.get("MIFX_DP_FORK_ONCE", "1") != "0"


@dataclass
class _Bucket:
    params: list
    numel: int
    buf: torch.Tensor
    offsets: list = field(default_factory=list)
    pending: int = 0
    work: object = None
    ready: set = field(default_factory=set)


class DataParallel:
    """Wraps a module; call `finish()` after `loss.backward()` and before `optimizer.step()`."""

    def __init__(self, module: torch.nn.Module, process_group=None, bucket_cap_mb: float = 32.0,
                 wire_dtype: torch.dtype | None = None, broadcast_init: bool = True, average: bool = True,
                 grad_as_bucket_view: bool = False, exchange: str = "rccl", force: bool = False):
        """force: run the hooks and the exchange even on a one-rank group (a measurement of the data-parallel
        machinery's own cost on one GPU: the exchange of a one-rank group is a copy through the peer buffers)."""
        if grad_as_bucket_view and wire_dtype is not None:
            raise ValueError("gradients as bucket views need the parameters' own dtype on the wire")
        if exchange not in ("rccl", "ipc", "auto"):
            raise ValueError(f"exchange: rccl, ipc or auto, not {exchange!r}")
        self.module = module
        self.views = bool(grad_as_bucket_view)
        self.pg = process_group if process_group is not None else (dist.group.WORLD if dist.is_initialized()
                                                                    else None)
        self.world = dist.get_world_size(self.pg) if self.pg is not None else 1
        self.active = self.world > 1 or (force and self.pg is not None)
        self.average = average
        self.wire_dtype = wire_dtype
        self._sync = True
        params = [p for p in module.parameters() if p.requires_grad]
        if broadcast_init and self.world > 1:
            with torch.no_grad():
                for p in list(module.parameters()) + list(module.buffers()):
                    dist.broadcast(p.data, src=dist.get_global_rank(self.pg, 0) if self.pg is not dist.group.WORLD
                                   else 0, group=self.pg)
        cap = int(bucket_cap_mb * 1024 * 1024)
        self.buckets: list[_Bucket] = []
        cur, cur_bytes = [], 0
        for p in reversed(params):
            nbytes = p.numel() * p.element_size()
            if cur and cur_bytes + nbytes > cap:
                self._add_bucket(cur)
                cur, cur_bytes = [], 0
            cur.append(p)
            cur_bytes += nbytes
        if cur:
            self._add_bucket(cur)
        self._where = {}
        for bi, b in enumerate(self.buckets):
            for pi, p in enumerate(b.params):
                self._where[p] = (bi, pi)
        dev = params[0].device if params else torch.device("cpu")
        self._comm_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self._next = 0  # the next bucket to launch (buckets launch in order)
        # coalesced deferred flushes: the smallest grouped launch worth issuing before the end of the backward
        # (workgroups), MIFX_DP_FLUSH_MIN_WG. Default: never -- ONE grouped flush after the backward, then the bucket
        # exchanges. Measured on the ResNet-50 B=256 step forced onto one rank (profiles/resnet_dp_census_r6.md,
        # profiles/resnet_dp_flush_r6.md): one flush + exchanges after the backward 21.46 ms vs 23.10 ms for a flush
        # and an overlapped exchange per bucket (0), whose small grouped launches leave CUs idle (+0.9 ms of flush
        # time), and 21.92 / 22.23 ms for thresholds 2048 / 1024 (runs of buckets flushed together, their exchanges
        # overlapping the rest of the backward: on one rank the exchange is cheap, the extra launches are not).
        self.flush_min_wgs = int(os.environ.get("MIFX_DP_FLUSH_MIN_WG", str(1 << 40)))
        self._flush_last = os.environ.get("MIFX_DP_FLUSH_LAST", "0") == "1"  # (diagnostic switches, A/B)
        self._launch_late = os.environ.get("MIFX_DP_LAUNCH_LATE", "0") == "1"
        self.deferred = False  # set by a trainer whose backward records weight gradients for grouped flushes
        self._ipc = None
        if exchange != "rccl" and self.active:
            self._ipc = self._open_ipc(dev, required=exchange == "ipc")
        self.exchange = "ipc" if self._ipc is not None else ("rccl" if self.active else "none")
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in params] if self.active else []
        if self.views:
            self.zero_grad()

    def _open_ipc(self, dev, required: bool):
        """The fp32 peer-memory all-reduce sized for the largest bucket, or None (auto: RCCL) when it cannot be set up
        on every rank (the setup agrees over the group, so all ranks take the same exchange)."""
        ok = dev.type == "cuda" and self.world <= 8 and all(b.buf.dtype == torch.float32 and b.numel % 2 == 0
                                                             for b in self.buckets)
        flags = [None] * self.world
        dist.all_gather_object(flags, bool(ok), group=self.pg)
        if not all(flags):
            if required:
                raise RuntimeError("DataParallel exchange='ipc' needs CUDA fp32 buckets of even size on <= 8 ranks")
            return None
        from .tp_ipc import IpcAllReduce

        try:
            # split waits: the exchange runs on a side stream beside the backward's whole-CU GEMM kernels (the
            # deferred weight-gradient flushes), so no exchange workgroup may spin on a late peer
            return IpcAllReduce(self.pg, dev, max(b.numel for b in self.buckets), dtype=torch.float32,
                                waiters=os.environ.get("MIFX_DP_WAITERS", "1") != "0")
        except RuntimeError:
            if required:
                raise
            return None

    def _view(self, b: _Bucket, pi: int) -> torch.Tensor:
        p, off = b.params[pi], b.offsets[pi]
        return b.buf[off:off + p.numel()].as_strided(p.shape, p.stride())

    def zero_grad(self) -> None:
        """(grad_as_bucket_view) zero every bucket and (re)attach each param.grad as its bucket view."""
        for b in self.buckets:
            b.buf.zero_()
            for pi, p in enumerate(b.params):
                g = p.grad
                if g is None or g.data_ptr() != b.buf.data_ptr() + b.offsets[pi] * b.buf.element_size():
                    p.grad = self._view(b, pi)

    def _add_bucket(self, params: list) -> None:
        n = sum(p.numel() for p in params)
        dt = self.wire_dtype or params[0].dtype
        b = _Bucket(params=list(params), numel=n, buf=torch.empty(n, dtype=dt, device=params[0].device))
        off = 0
        for p in params:
            b.offsets.append(off)
            off += p.numel()
        b.pending = len(params)
        self.buckets.append(b)

    # ---- hooks ------------------------------------------------------------------------------
    def _on_grad(self, p: torch.Tensor) -> None:
        if p.grad is None:
            return
        bi, pi = self._where[p]
        b = self.buckets[bi]
        off = b.offsets[pi]
        view = b.buf[off:off + p.numel()]
        if self.views and p.grad.data_ptr() != view.data_ptr():
            # views mode assumes p.grad IS the bucket view; something replaced it (optimizer.zero_grad() with
            # set_to_none, a weight released for a deferred flush that the flush did not take): copy the fresh
            # gradient into the bucket and re-attach the view -- in the parameter's own layout (channels_last), so the
            # all-reduced bucket and the gradient the optimizer reads stay the same memory, element for element. Also
            # under no_sync: the bucket must hold what the later (eager) exchange reduces.
            v = self._view(b, pi)
            v.copy_(p.grad)
            p.grad = v
        if not self._sync or pi in b.ready:
            return
        b.ready.add(pi)
        if not self.views:
            view.copy_(p.grad.reshape(-1))
        if len(b.ready) == len(b.params):
            self._complete_ready()

    def _complete_ready(self) -> None:
        """A bucket just completed. Without deferred products: launch every complete bucket in order. With them: the
        run of complete, unlaunched buckets (from the next one in launch order) is flushed in ONE grouped launch and
        their exchanges launched right after -- but only once the run's recorded work fills the GPU (flush_min_wgs
        workgroups): a bucket of few, small products (the last stage's weights hold few output tiles) flushed alone
        leaves most CUs idle, which measured +0.9 ms over one flush per step in the ResNet-50 DP step
        (profiles/resnet_dp_census_r6.md). Later flushes still overlap the earlier buckets' exchanges."""
        run = []
        for b in self.buckets[self._next:]:
            if len(b.ready) != len(b.params):
                break
            run.append(b)
        if not run:
            return
        if self.deferred:
            from ..ops import gemm as hg

            pend = hg.pending_weights()
            mine = [p for b in run for p in b.params if id(p) in pend]
            last = run[-1] is self.buckets[-1]  # every bucket complete: flush now, whatever the size
            if mine:
                if hg.pending_work(mine) < self.flush_min_wgs and not (last and self._flush_last):
                    return  # wait for more buckets (finish() flushes whatever is left)
                hg.flush_weight_grads(mine)
        if not self._launch_late:
            self._launch_ready()

    def _flush_deferred(self, b: _Bucket) -> None:
        """Deferred weight gradients (mifx.ops.gemm.deferred_weight_grads): the bucket's recorded dW products as one
        grouped launch on the compute stream, written straight into the bucket views (finish(): every remaining
        bucket's at once)."""
        self._flush_many([b])

    def _flush_many(self, buckets) -> None:
        if not self.deferred:
            return
        from ..ops import gemm as hg

        pend = hg.pending_weights()
        mine = [p for b in buckets for p in b.params if id(p) in pend]
        if mine:
            hg.flush_weight_grads(mine)

    def grad_view(self, p: torch.Tensor) -> torch.Tensor | None:
        """A fresh view of p's slot in its bucket (bucket-view mode), the placeholder a deferred weight gradient is
        written into; None for parameters this wrapper does not own."""
        w = self._where.get(p)
        if w is None or not self.views:
            return None
        return self._view(self.buckets[w[0]], w[1])

    def release_grads_for_defer(self) -> None:
        """Before a backward with deferred weight gradients, instead of zero_grad(): drop every parameter's .grad (the
        bucket memory stays), so autograd adopts the bucket view handed out as the placeholder of a deferred product
        (grad_view) or as the output of a kernel that writes a parameter gradient itself (BatchNorm's dgamma / dbeta,
        mifx.ops.gemm.grad_destination) -- the gradient is WRITTEN into the bucket, with no memset of the buckets and no
        zero-fill + add. A gradient produced elsewhere is copied into the bucket by the post-accumulate hook; a parameter
        that gets no gradient has its slot zeroed by finish()."""
        for b in self.buckets:
            for p in b.params:
                p.grad = None

    def _launch_ready(self) -> None:
        """Launch every complete bucket from the next one in bucket order on (one fork of the communication stream
        for all of them: the compute stream has not moved in between)."""
        fork = True
        while self._next < len(self.buckets):
            b = self.buckets[self._next]
            if len(b.ready) != len(b.params):
                return
            self._launch(b, fork or not _FORK_ONCE)
            fork = False

    def _launch(self, b: _Bucket, fork: bool = True) -> None:
        assert b is self.buckets[self._next], "buckets launch in order"
        self._next += 1
        if self._comm_stream is not None and _COMM_DIAG == "copy":  # diagnostic: a plain in-place round trip
            if getattr(self, "_diag_tmp", None) is None:
                self._diag_tmp = torch.empty(max(bb.numel for bb in self.buckets), dtype=b.buf.dtype,
                                             device=b.buf.device)
            self._comm_stream.wait_stream(torch.cuda.current_stream(b.buf.device))
            with torch.cuda.stream(self._comm_stream):
                t = self._diag_tmp[:b.numel]
                t.copy_(b.buf)
                b.buf.copy_(t)
            b.work = "ipc"
            return
        if self._comm_stream is not None and self._ipc is not None and _COMM_DIAG == "main":
            self._ipc.all_reduce(b.buf, out=b.buf, scale=1.0 / self.world if self.average else 1.0)
            b.work = "ipc"
        elif self._comm_stream is not None:
            cur = torch.cuda.current_stream(b.buf.device)
            if fork:
                self._comm_stream.wait_stream(cur)
            with torch.cuda.stream(self._comm_stream):
                if self._ipc is not None:  # averaged in the kernel; stream-ordered, graph-capturable
                    self._ipc.all_reduce(b.buf, out=b.buf, scale=1.0 / self.world if self.average else 1.0)
                    b.work = "ipc"
                else:
                    b.work = dist.all_reduce(b.buf, group=self.pg, async_op=True)
            if _COMM_DIAG == "join":
                cur.wait_stream(self._comm_stream)
        else:
            b.work = dist.all_reduce(b.buf, group=self.pg, async_op=True)

    # ---- public API ---------------------------------------------------------------------------
    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate gradients locally (e.g. micro-batches) without communicating."""
        old, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = old

    def __call__(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    def finish(self) -> None:
        """Complete all bucket all-reduces (launching buckets whose params got no gradient) and write
        the averaged gradients back into `param.grad`."""
        if not self.active or not self._sync:
            return
        self._flush_many(self.buckets[self._next:])  # ONE grouped launch for every bucket not launched yet
        for b in self.buckets[self._next:]:  # (in order: an incomplete bucket holds back its successors)
            if self.views:  # released gradients that never arrived: a zero slot (see release_grads_for_defer)
                for pi, p in enumerate(b.params):
                    if p.grad is None:
                        v = self._view(b, pi)
                        v.zero_()
                        p.grad = v
            if b.work is None and not self.views:  # unused params this step: contribute zeros for them
                for pi, p in enumerate(b.params):
                    if pi not in b.ready:
                        off = b.offsets[pi]
                        if p.grad is None:
                            b.buf[off:off + p.numel()].zero_()
                        else:
                            b.buf[off:off + p.numel()].copy_(p.grad.reshape(-1))
        # (views: unused params' bucket views are still zero)
        for i, b in enumerate(self.buckets[self._next:]):  # one fork of the communication stream for all of them
            self._launch(b, i == 0 or not _FORK_ONCE)
        self._next = 0
        cur = torch.cuda.current_stream(self.buckets[0].buf.device) if self._comm_stream is not None else None
        scale = 1.0 / self.world if self.average else 1.0
        if self._ipc is not None:  # the kernels averaged in place; join the side stream
            cur.wait_stream(self._comm_stream)
            for b in self.buckets:
                if not self.views:
                    for pi, p in enumerate(b.params):
                        off = b.offsets[pi]
                        g = b.buf[off:off + p.numel()].view_as(p).to(p.dtype)
                        if p.grad is None:
                            p.grad = g.clone()
                        else:
                            p.grad.copy_(g)
                b.work, b.ready = None, set()
            return
        for b in self.buckets:
            b.work.wait()
            if cur is not None:
                cur.wait_stream(self._comm_stream)
            if self.views:  # param.grad are views of the bucket: average in place, nothing to copy back
                if scale != 1.0:
                    b.buf.mul_(scale)
                b.work, b.ready = None, set()
                continue
            for pi, p in enumerate(b.params):
                off = b.offsets[pi]
                g = b.buf[off:off + p.numel()].view_as(p).to(p.dtype)
                if p.grad is None:
                    p.grad = g.mul(scale)
                else:
                    p.grad.copy_(g).mul_(scale)
            b.work, b.ready = None, set()

    step_ready = finish

    def check(self) -> None:
        """Raise if the peer-memory exchange timed out on this rank. Its error flag is sticky: every later exchange
        poisons its bucket with NaN instead of hanging, so a caller must check at each host synchronisation point
        (after warmup, after timed steps, before writing a checkpoint) rather than train on or save NaN weights."""
        if self._ipc is not None:
            self._ipc.check()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def allreduce_flat_(t: torch.Tensor, group=None, average: bool = True) -> torch.Tensor:
    """In-place all-reduce of one flat tensor (the latency-bound small-gradient path, e.g. W&D's
    ≈120 KB gradient: one collective per step is the minimum)."""
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
        if average:
            t.div_(dist.get_world_size(group))
    return t
