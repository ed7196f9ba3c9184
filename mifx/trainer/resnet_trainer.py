"""ResNet-50 image-classification trainer (BASELINE config 5): data-parallel over the node's MI355X (one process per
GPU), HBM-resident uint8 dataset with the fused crop/flip/normalize HIP kernel, bf16 channels_last. The convolutions
run on the hand-written implicit-GEMM kernel (csrc/gemm8.hip, mifx.ops.conv1x1 / conv3x3) with BatchNorm statistics,
BatchNorm-backward sums and residual adds in its epilogues; weight gradients are deferred to grouped launches
(mifx.ops.gemm.deferred_weight_grads); SGD + Nesterov momentum with linear warmup is one fused multi-tensor kernel
(csrc/sgd.hip). What MIOpen still runs is listed in README.md.

On the GPU the step is captured into hipGraphs after `graph_warmup` eager steps (graph=True, the default there):
graph A = gradient zeroing + every micro-batch's input kernel, forward and backward (the step counter, learning rate
and sample indices are device tensors written before each replay). Data-parallel with the peer-memory exchange
(DataParallel exchange="ipc", the default on the GPU: MIFX_DP_EXCHANGE=auto|ipc|rccl) the bucket all-reduces are
kernels launched on the side stream as each bucket's gradients complete -- overlapped with the rest of the backward
and captured with it -- and SGD follows in the same graph: ONE graph per step, nothing eager between. With the RCCL
exchange the all-reduces run eagerly between graph A and graph B (SGD). One graph without data parallelism.

`python -m torch.distributed.run --nproc-per-node 8 -m mifx.trainer.resnet_trainer` prints images/sec."""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

from ..models.resnet import resnet50_v2
from ..ops.bn_relu import defer_batch_counts
from ..ops.image_ops import IMAGENET_MEAN, IMAGENET_STD, crop_flip_normalize
from ..parallel import dist as mdist
from ..parallel.ddp import DataParallel
from ..utils.meter import heartbeat


def synthetic_imagenet(n: int, size: int = 256, classes: int = 1000, seed: int = 0, device="cpu"):
    """uint8 NHWC images with a weak class signal (per-class mean colour) + int64 labels."""
    g = torch.Generator(device=device).manual_seed(seed)
    labels = torch.randint(0, classes, (n,), generator=g, device=device)
    base = (torch.arange(classes, device=device)[:, None] * torch.tensor([37, 91, 151], device=device)) % 200
    imgs = torch.randint(0, 56, (n, size, size, 3), generator=g, device=device, dtype=torch.uint8)
    imgs += base[labels].to(torch.uint8)[:, None, None, :]
    return imgs, labels


class ResNetTrainer:
    def __init__(self, batch: int, device, images: torch.Tensor, labels: torch.Tensor, num_classes: int = 1000,
                 lr: float = 0.1, momentum: float = 0.9, weight_decay: float = 5e-5, warmup_steps: int = 100,
                 process_group=None, mean=IMAGENET_MEAN, std=IMAGENET_STD, seed: int = 0, crop: int = 224,
                 accum_steps: int = 1, graph: bool | None = None, graph_warmup: int = 2, force_dp: bool = False):
        """batch: examples per micro-batch per replica; accum_steps micro-batches (each with its own BatchNorm
        statistics) are summed into one update. A data-parallel step over W ranks trains on W x accum_steps x batch
        examples: the global sample of the step is drawn from (seed, step) and rank r takes micro-batches
        r accum_steps .. (r + 1) accum_steps - 1 of it, so W ranks at accum 1 compute the same update as one
        process at accum W (up to fp32 summation order)."""
        self.device = torch.device(device)
        self.batch, self.crop, self.seed = batch, crop, seed
        self.accum = max(1, int(accum_steps))
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.rank = torch.distributed.get_rank(process_group) if process_group is not None else 0
        torch.manual_seed(seed)
        self.model = resnet50_v2(num_classes).to(self.device).to(memory_format=torch.channels_last)
        self._bn_count = defer_batch_counts(self.model)  # one counter kernel per forward, not one per BatchNorm
        exch = os.environ.get("MIFX_DP_EXCHANGE", "auto") if self.device.type == "cuda" else "rccl"
        self.dp = DataParallel(self.model, process_group, grad_as_bucket_view=True, exchange=exch,
                               bucket_cap_mb=float(os.environ.get("MIFX_DP_BUCKET_MB", "16")), force=force_dp) \
            if process_group is not None else None
        decay = [p for n, p in self.model.named_parameters() if p.ndim > 1]
        no_decay = [p for n, p in self.model.named_parameters() if p.ndim <= 1]
        self.opt = torch.optim.SGD([{"params": decay, "weight_decay": weight_decay},
                                    {"params": no_decay, "weight_decay": 0.0}], lr=lr, momentum=momentum,
                                   nesterov=True)
        # bf16 images of the GEMM-shaped convolutions' weights, refreshed in one launch at the start of every step
        self.prep = None
        if self.device.type == "cuda" and os.environ.get("MIFX_WEIGHT_PREP", "1") != "0":
            from ..ops.weight_prep import WeightPrep

            ws = [m.weight for m in self.model.modules() if isinstance(m, torch.nn.Conv2d) and m.groups == 1
                  and (m.kernel_size == (1, 1) or (m.kernel_size == (3, 3) and m.in_channels >= 64))
                  and WeightPrep.supported(m.weight)]
            self.prep = WeightPrep(ws) if ws else None
        self.base_lr, self.warmup = lr, warmup_steps
        self.images, self.labels = images.to(self.device), labels.to(self.device)
        self.mean, self.std = mean, std
        self.step_idx = 0
        self.amp = self.device.type == "cuda"
        self.defer_dw = self.amp and os.environ.get("MIFX_DEFER_DW", "1") != "0"
        if self.amp:  # MIOpen find: benchmark the solvers once per conv shape, then reuse (+12% measured)
            torch.backends.cudnn.benchmark = True
        # captured steps (GPU): eager for the first graph_warmup steps (MIOpen find, momentum buffers), then graphs
        self.use_graph = (self.device.type == "cuda") if graph is None else (bool(graph) and self.device.type == "cuda")
        self.graph_warmup = max(1, int(graph_warmup))
        self._gA = self._gB = None
        self._eager_done = 0  # eager steps since construction / restore (the capture needs warm MIOpen solvers)
        if self.use_graph:
            n = self.world * self.accum * self.batch
            self._idx_dev = torch.zeros(n, dtype=torch.int64, device=self.device)
            self._step_dev = torch.zeros(1, dtype=torch.int64, device=self.device)
            self._neg_lr = torch.zeros((), dtype=torch.float32, device=self.device)  # 0-dim: a foreach scalar

    def _count_forward(self) -> None:
        if self._bn_count is not None and self.model.training:
            self._bn_count.add_(1)

    def _lr(self) -> float:
        return self.base_lr * min(1.0, (self.step_idx + 1) / max(1, self.warmup))

    def _step_indices(self) -> torch.Tensor:
        """The global sample of this step ([world * accum * batch], from (seed, step) on a host generator: the same
        on every rank and device)."""
        g = torch.Generator().manual_seed(self.seed * 1000003 + self.step_idx)
        return torch.randint(0, len(self.labels), (self.world * self.accum * self.batch,), generator=g)

    def step(self) -> torch.Tensor:
        if self.use_graph and self._eager_done >= self.graph_warmup:
            return self._graph_step()
        self._eager_done += 1
        return self._eager_step()

    def _eager_step(self) -> torch.Tensor:
        glob = self._step_indices()
        for pg in self.opt.param_groups:
            pg["lr"] = self._lr()
        if self.dp is not None:
            if self.defer_dw:  # gradients WRITTEN into the bucket views (deferred products, BatchNorm): no memset
                self.dp.deferred = True
                self.dp.release_grads_for_defer()
            else:
                self.dp.zero_grad()  # the bucket buffers ARE the gradients (views): one memset per bucket
        else:
            self.opt.zero_grad(set_to_none=True)
        total = 0.0
        if self.prep is not None:
            self.prep.refresh()
        for m in range(self.accum):
            mb = self.rank * self.accum + m
            idx = glob[mb * self.batch:(mb + 1) * self.batch].to(self.device)
            x = crop_flip_normalize(self.images, idx, (self.crop, self.crop), True, self.seed, self.step_idx,
                                    self.mean, self.std, torch.bfloat16 if self.amp else torch.float32)
            y = self.labels[idx]
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                loss = F.cross_entropy(self.model(x).float(), y) / self.accum
            self._count_forward()
            last = m == self.accum - 1
            self._backward(loss, last)
            total = total + loss.detach()
        if self.dp is not None:
            self.dp.finish()
        self.opt.step()
        self.step_idx += 1
        return total

    def _backward(self, loss: torch.Tensor, last: bool, sync: bool = True) -> None:
        """One micro-batch's backward. Deferred weight gradients (the GEMM-shaped convolutions' dW recorded during the
        backward and run as grouped split-K launches of csrc/gemm8.hip): without data parallelism ONE flush after the
        backward; with it, each bucket's products are flushed the moment the bucket's last gradient is accumulated,
        straight into the bucket views, and its exchange launched right after -- so the exchanges overlap the rest of
        the backward and the later flushes. Micro-batches before the last accumulate locally (no_sync, one flush)."""
        dp = self.dp if sync else None
        if not self.defer_dw:
            if dp is not None and not last:
                with dp.no_sync():
                    loss.backward()
            else:
                loss.backward()
            return
        from ..ops import gemm as hg

        if dp is None or not last:
            ctx = dp.no_sync() if dp is not None else contextlib.nullcontext()
            with ctx, hg.deferred_weight_grads(view_of=self.dp.grad_view if self.dp is not None else None):
                loss.backward()
            hg.flush_weight_grads()
            return
        with hg.deferred_weight_grads(view_of=dp.grad_view):
            loss.backward()  # the DataParallel hooks flush and exchange bucket by bucket
        hg.flush_weight_grads()  # (the bf16 products of non-bucketed weights, if any)

    # ---------------------------------------------------------------- captured step
    def _graph_step(self) -> torch.Tensor:
        glob = self._step_indices()
        if self._gA is None:
            self._capture()
        self._idx_dev.copy_(glob)
        self._step_dev.fill_(self.step_idx)
        self._neg_lr.fill_(-self._lr())
        for pg in self.opt.param_groups:
            pg["lr"] = self._lr()  # (kept current for checkpoints / eager fallbacks)
        self._gA.replay()
        if self._gB is not None:
            self.dp.finish()  # bucket all-reduces (RCCL) in place on the gradient views, averaged
            self._gB.replay()
        self.step_idx += 1
        return self._static_loss

    def _fwd_bwd_captured(self) -> torch.Tensor:
        defer = self.defer_dw
        if self.dp is not None:
            if defer:  # gradients written into the bucket views (see _eager_step)
                self.dp.deferred = True
                self.dp.release_grads_for_defer()
            else:
                for b in self.dp.buckets:  # param.grad are views of these
                    b.buf.zero_()
        elif defer:
            # gradients produced inside the graph (its private pool: the same addresses on every replay, which the
            # captured SGD reads); the deferred weight-gradient flush then overwrites instead of zero-fill + add
            for p in self.model.parameters():
                p.grad = None
        else:
            torch._foreach_zero_([p.grad for p in self.model.parameters() if p.grad is not None])
        total = None
        if self.prep is not None:
            self.prep.refresh()
        in_graph = self.dp is not None and self.dp.exchange == "ipc"  # the exchange captures with the backward
        ctx = self.dp.no_sync() if self.dp is not None and not in_graph else contextlib.nullcontext()
        with ctx:
            for m in range(self.accum):
                mb = self.rank * self.accum + m
                idx = self._idx_dev[mb * self.batch:(mb + 1) * self.batch]
                x = crop_flip_normalize(self.images, idx, (self.crop, self.crop), True, self.seed, 0, self.mean,
                                        self.std, torch.bfloat16 if self.amp else torch.float32,
                                        step_dev=self._step_dev)
                y = self.labels[idx]
                with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                    loss = F.cross_entropy(self.model(x).float(), y) / self.accum
                self._count_forward()
                # the same backward as the eager steps; the exchange captures with it only on the ipc path (RCCL:
                # the whole graph runs under no_sync and the bucket all-reduces run eagerly between the graphs)
                self._backward(loss, m == self.accum - 1, sync=in_graph)
                total = loss.detach() if total is None else total + loss.detach()
        if in_graph:
            self.dp.finish()  # joins the side stream: every bucket exchanged and averaged
        return total

    def _sgd_prepare(self) -> None:
        """Tables of the fused multi-tensor SGD (csrc/sgd.hip, one launch instead of 14 foreach passes), built
        before a capture (they are host-to-device copies). MIFX_SGD_FUSED=0, or groups with different momentum
        settings, keep the foreach update."""
        self._sgd_tab = None
        if os.environ.get("MIFX_SGD_FUSED", "1") == "0" or not self.device.type == "cuda":
            return
        groups = self.opt.param_groups
        if len({(g["momentum"], g["dampening"], g["nesterov"]) for g in groups}) != 1:
            return
        from ..ops import _lib
        from ..ops.sgd import FusedSGDTables

        if not _lib.available("sgd"):
            return
        params, bufs, wds = [], [], []
        for g in groups:
            for p in g["params"]:
                if not p.requires_grad:
                    continue
                params.append(p)
                bufs.append(self.opt.state[p]["momentum_buffer"])
                wds.append(g["weight_decay"])
        try:
            self._sgd_tab = FusedSGDTables(params, bufs, wds)
        except ValueError:
            self._sgd_tab = None

    @torch.no_grad()
    def _sgd_captured(self) -> None:
        """torch.optim.SGD's update (weight decay, momentum, Nesterov; its own momentum buffers) with the learning
        rate read from a device tensor, so a replayed graph follows the warmup schedule."""
        tab = getattr(self, "_sgd_tab", None)
        if tab is not None:
            grads = [p.grad for p in tab.params]  # (with deferred weight gradients: produced inside this capture)
            if tab.grads_ok(grads):
                tab.set_grads(grads)
                g0 = self.opt.param_groups[0]
                tab.step(self._neg_lr, g0["momentum"], g0["dampening"], g0["nesterov"])
                return
            self._sgd_tab = None  # a gradient missing or laid out unlike its parameter: the foreach update
        for group in self.opt.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            grads = [p.grad for p in params]
            bufs = [self.opt.state[p]["momentum_buffer"] for p in params]
            wd, mom, damp = group["weight_decay"], group["momentum"], group["dampening"]
            if wd:
                grads = torch._foreach_add(grads, params, alpha=wd)
            torch._foreach_mul_(bufs, mom)
            torch._foreach_add_(bufs, grads, alpha=1 - damp)
            if group["nesterov"]:
                upd = torch._foreach_add(grads, bufs, alpha=mom)
            else:
                upd = [b.clone() for b in bufs]
            torch._foreach_mul_(upd, self._neg_lr)
            torch._foreach_add_(params, upd)

    def _capture(self) -> None:
        if any("momentum_buffer" not in self.opt.state.get(p, {}) for p in self.model.parameters()
               if p.requires_grad):
            raise RuntimeError("capture needs the SGD momentum buffers of an eager step first")
        self._sgd_prepare()
        torch.cuda.synchronize(self.device)
        self._gA = torch.cuda.CUDAGraph()
        one = self.dp is None or self.dp.exchange == "ipc"
        with torch.cuda.graph(self._gA):
            self._static_loss = self._fwd_bwd_captured()
            if one:
                self._sgd_captured()
        if not one:
            self._gB = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self._gB):
                self._sgd_captured()

    def check(self) -> None:
        """Raise if the data-parallel peer-memory exchange timed out on this rank (sticky: the later steps' buckets
        are NaN, so nothing trained since may be reported or saved)."""
        if self.dp is not None:
            self.dp.check()

    # ---------------------------------------------------------------- checkpoint / resume
    def state_dict(self) -> dict:
        """Weights, BatchNorm running statistics, the SGD momentum buffers and the step (flat tensor dict)."""
        # (clone: the BatchNorm counters are views of one tensor, which safetensors would refuse as shared memory)
        sd = {f"model.{k}": v.detach().clone() for k, v in self.model.state_dict().items()}
        for i, p in enumerate(self.model.parameters()):
            buf = self.opt.state.get(p, {}).get("momentum_buffer")
            if buf is not None:
                sd[f"opt.momentum.{i}"] = buf.detach().contiguous()
        sd["step"] = torch.tensor([self.step_idx], dtype=torch.int64)
        return sd

    def load_state_dict(self, sd: dict) -> None:
        self.model.load_state_dict({k[6:]: v for k, v in sd.items() if k.startswith("model.")})
        for i, p in enumerate(self.model.parameters()):
            v = sd.get(f"opt.momentum.{i}")
            if v is not None:
                self.opt.state[p]["momentum_buffer"] = v.to(device=p.device, dtype=p.dtype).clone() \
                    .contiguous(memory_format=torch.channels_last if p.ndim == 4 else torch.contiguous_format)
        self.step_idx = int(sd["step"][0])
        self._gA = self._gB = None  # the graphs captured the old momentum buffers: re-capture after warm steps
        self._eager_done = 0

    def save_checkpoint(self, model_dir: str, keep: int = 1) -> str:
        import glob as _glob
        import os

        from safetensors.torch import save_file

        self.check()  # never write weights trained on a failed exchange
        os.makedirs(model_dir, exist_ok=True)
        path = os.path.join(model_dir, f"ckpt-{self.step_idx}.safetensors")
        save_file({k: v.cpu().contiguous() for k, v in self.state_dict().items()}, path)
        old = sorted(_glob.glob(os.path.join(model_dir, "ckpt-*.safetensors")),
                     key=lambda q: int(q.rsplit("-", 1)[1].split(".")[0]))
        for q in old[:-max(1, keep)]:
            os.remove(q)
        return path

    @staticmethod
    def latest_checkpoint(model_dir: str) -> str | None:
        import glob as _glob
        import os

        c = sorted(_glob.glob(os.path.join(model_dir, "ckpt-*.safetensors")),
                   key=lambda q: int(q.rsplit("-", 1)[1].split(".")[0]))
        return c[-1] if c else None

    def restore(self, path: str) -> None:
        from safetensors.torch import load_file

        self.load_state_dict(load_file(path))

    @torch.no_grad()
    def evaluate(self, images: torch.Tensor, labels: torch.Tensor, batch: int = 256) -> float:
        self.model.eval()
        correct = 0
        for s in range(0, len(labels), batch):
            idx = torch.arange(s, min(s + batch, len(labels)), device=self.device)
            x = crop_flip_normalize(images.to(self.device), idx, (self.crop, self.crop), False, 0, 0, self.mean,
                                    self.std, torch.bfloat16 if self.amp else torch.float32)
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                correct += int((self.model(x).argmax(1) == labels[s:s + batch].to(self.device)).sum())
        self.model.train()
        return correct / len(labels)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256, help="per GPU")
    ap.add_argument("--images", type=int, default=2048, help="HBM-resident images per GPU")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--deterministic", action="store_true",
                    help="MIOpen deterministic convolution solvers: bit-reproducible steps (the default bf16 solvers "
                         "are not run-to-run reproducible, measured in round 2, profiles/archive/resnet_determinism_r2s3.txt). Diagnostic only: "
                         "measured 13.7 s/step at B=256 on one MI355X vs 26.5 ms with the default solvers")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of the captured hipGraph step")
    a = ap.parse_args(argv)
    if a.deterministic:
        torch.backends.cudnn.deterministic = True
    env = mdist.init()
    # MIFX_SHARED_GPU=1 (with MIFX_DIST_BACKEND=gloo): the multi-rank flow rehearsed with every rank on cuda:0
    local = 0 if os.environ.get("MIFX_SHARED_GPU") == "1" else env.local_rank
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    imgs, labels = synthetic_imagenet(a.images, seed=env.rank, device=dev)
    force = os.environ.get("MIFX_DP_FORCE") == "1" and env.world_size == 1
    if force:  # the data-parallel machinery on one rank (hooks, bucket exchange): its overhead, measured
        import socket

        with socket.socket() as s_:
            s_.bind(("127.0.0.1", 0))
            port = s_.getsockname()[1]
        torch.distributed.init_process_group("nccl" if dev.type == "cuda" else "gloo",
                                             init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    pg = torch.distributed.group.WORLD if env.world_size > 1 or force else None
    tr = ResNetTrainer(a.batch, dev, imgs, labels, process_group=pg, warmup_steps=10, graph=not a.no_graph,
                       force_dp=force)
    for i in range(a.warmup):  # first steps include MIOpen solver search/compile: report progress
        t1 = time.perf_counter()
        with heartbeat("resnet warmup"):
            tr.step()
            if dev.type == "cuda":
                torch.cuda.synchronize()
        if env.rank == 0:
            print(f"[resnet] warmup step {i + 1}/{a.warmup}: {time.perf_counter() - t1:.2f}s", file=sys.stderr,
                  flush=True)
    tr.check()  # a timed-out exchange during warmup fails the run here, outside the timed region
    mdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = tr.step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    mdist.barrier()
    dt = mdist.max_over_ranks(time.perf_counter() - t0)
    tr.check()  # ... and during the timed steps: never report the throughput of NaN buckets
    if env.rank == 0:
        print(json.dumps({"metric": "ResNet-50 training images/sec (whole node)",
                          "value": a.batch * env.world_size * a.steps / dt, "unit": "images/s",
                          "n_gpus": env.world_size, "batch_per_gpu": a.batch, "ms_per_step": 1e3 * dt / a.steps,
                          "loss": float(loss), "dtype": "bf16", "data": "synthetic ImageNet-shaped (HBM-resident)",
                          "parallelism": f"dp{env.world_size}", "hipgraph": tr.use_graph,
                          "dp_exchange": tr.dp.exchange if tr.dp is not None else "none",
                          "graphs_per_step": 0 if not tr.use_graph else (2 if tr._gB is not None else 1),
                          "sgd": "fused" if getattr(tr, "_sgd_tab", None) is not None else "foreach",
                          "deterministic": bool(torch.backends.cudnn.deterministic)}), flush=True)
    mdist.shutdown()


if __name__ == "__main__":
    main()
