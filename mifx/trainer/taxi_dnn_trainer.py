"""Trainer for the KFP taxi DNN (`mifx.models.taxi_dnn`): HIP gather/scatter kernels on GPU,
PyTorch autograd + TF-semantics Adagrad on CPU (the numerics oracle).

Reference: dnntrainer component (`taxi-cab-classification-pipeline.py:117-126`): Adagrad lr 0.1,
hidden 1500, 3,000 steps, binary head; TF's Adagrad starts accumulators at 0.1."""
from __future__ import annotations

import numpy as np
import torch

from ..models.taxi_dnn import TaxiDNN
from .optim import TFAdagrad


class TaxiDNNTrainer:
    """On the GPU a step is 5 HIP launches with no host work: the batch is selected on the device from the
    HBM-resident records through a device step counter (advanced by the optimizer kernel), and the sparse Adagrad
    deduplicates rows in-kernel (no sort/unique, whose dynamic output size synchronised the host every step). So
    the step is captured once into hipGraphs -- one step and `steps_per_graph` consecutive steps -- and replayed
    (`graph=False`: eager launches of the same kernels).

    Data parallel (`process_group`, one rank per GPU): the 6170 x 1500 first layer makes the DENSE gradient 37 MB
    (the bandwidth-relevant case), but a step touches only batch x 13 of its 6,167 sparse rows. So
    the ranks exchange the step's per-example backward state instead -- activations, hidden-layer gradient dz,
    dense inputs, dlogit and the W1 row ids: B x (2H + D + 1 + F) floats, ~0.4 MB per rank at B=32 -- with ONE
    all-gather, and every rank runs the sparse + dense Adagrad kernels over the gathered global batch (rank-major =
    the global batch's example order). That is bit-identical to one process at batch world x B (same kernels, same
    summation order) for ~1/100 of the bytes a dense all-reduce would move over xGMI. The CPU path all-reduces
    dense gradients (mifx.parallel.ddp; TF-Adagrad leaves untouched rows unchanged under a zero gradient)."""

    def __init__(self, model: TaxiDNN | None = None, batch: int = 32, lr: float = 0.1, device="cpu",
                 initial_accumulator_value: float = 0.1, loss_reduction: str = "sum", native: bool | None = None,
                 graph: bool = True, steps_per_graph: int = 50, process_group=None, shuffle_seed: int = 0):
        """shuffle_seed: 0 = the records in stored order, else a fresh pseudo-random order every epoch, computed in
        the kernels' record selection (csrc/feed.h; the same order on the CPU path, mifx.data.shuffle). With a
        process group every rank keeps all records and trains on its slice of one global stream (stride
        world x batch, offset rank x batch), so the job equals one process at batch world x batch."""
        self.device = torch.device(device)
        self.model = (model or TaxiDNN()).to(self.device)
        self.batch, self.lr, self.loss_reduction = batch, lr, loss_reduction
        self.native = (self.device.type == "cuda") if native is None else native
        self.dense_row0 = self.model.cfg.sparse_rows
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        self.rank = torch.distributed.get_rank(process_group) if process_group is not None else 0
        self.feed = (self.world * batch, self.rank * batch, int(shuffle_seed) & (2**64 - 1))
        if self.world > 1:
            for p in self.model.parameters():  # identical initial replicas
                torch.distributed.broadcast(p.data, src=torch.distributed.get_global_rank(process_group, 0)
                                            if process_group is not torch.distributed.group.WORLD else 0,
                                            group=process_group)
        self.use_graph = bool(graph and self.native and self.world == 1)
        self.steps_per_graph = max(1, int(steps_per_graph))
        self.graph, self.graph_multi = None, None
        if self.native:
            from ..ops import embag_mlp

            self._k = embag_mlp
            if batch > embag_mlp.limits()["max_batch"]:
                raise ValueError(f"batch {batch} > {embag_mlp.limits()['max_batch']} (csrc/embag_mlp.hip kMaxList)")
            self.step_ctr = torch.zeros(1, dtype=torch.int64, device=self.device)
            p = {n: getattr(self.model, n) for n in ("W1", "b1", "w2", "b2")}
            self.params = {n: t.data for n, t in p.items()}
            self.accs = {n: torch.full_like(t, initial_accumulator_value) for n, t in self.params.items()}
            self.bufs = embag_mlp.make_buffers(batch, self.model.cfg.hidden, len(self.model.cfg.dense), self.device)
            if self.world > 1:
                self._init_exchange()
        else:
            self.opt = TFAdagrad(self.model.parameters(), lr=lr, initial_accumulator_value=initial_accumulator_value)
            if self.world > 1:
                from ..parallel.ddp import DataParallel

                self.dp = DataParallel(self.model, process_group, average=(loss_reduction == "mean"),
                                       broadcast_init=False)
        self.step_idx = 0
        self._last = float("nan")

    # ---------------------------------------------------------------- data parallel (sparse exchange)
    def _init_exchange(self) -> None:
        from ..ops import embag_mlp

        B, W = self.batch, self.world
        H, D, F = self.model.cfg.hidden, len(self.model.cfg.dense), len(self.model.cfg.sparse)
        Bg = B * W
        if Bg > embag_mlp.limits()["max_batch"]:
            raise ValueError(f"global batch {Bg} > {embag_mlp.limits()['max_batch']}")
        self.H, self.D, self.F, self.Bg = H, D, F, Bg
        self.gbufs = embag_mlp.make_buffers(Bg, H, D, self.device)
        self.g_rows = torch.empty(Bg, F, dtype=torch.int32, device=self.device)
        self.g_xd = torch.empty(Bg, D, device=self.device)
        self.C = 2 * H + D + 1
        # global batches of <= 64 take the kernels' per-example dense chunks (written by the forward/backward
        # launch): those travel too, so the update stays the single-process one
        self.direct = Bg <= 64
        self.NF = B * self.C + (B * (D + 2) * H if self.direct else 0)  # float32 words per rank
        # one BYTE buffer per rank: the float state, then the int32 W1 row ids -- a byte all-gather moves both
        # bit-exactly (no float copy ever touches the ids)
        self.L = 4 * (self.NF + B * F)
        self.send = torch.empty(self.L, dtype=torch.uint8, device=self.device)
        self.recv = torch.empty(W * self.L, dtype=torch.uint8, device=self.device)
        self.rec_idx = torch.zeros(B, dtype=torch.int64, device=self.device)

    def _all_gather(self) -> None:
        dist = torch.distributed
        if dist.get_backend(self.pg) == "nccl":
            dist.all_gather_into_tensor(self.recv, self.send, group=self.pg)
        else:  # gloo (CPU collectives; ranks sharing one GPU in rehearsals)
            parts = [torch.empty(self.L, dtype=torch.uint8) for _ in range(self.world)]
            dist.all_gather(parts, self.send.cpu(), group=self.pg)
            self.recv.copy_(torch.cat(parts))

    def _native_step_dp(self) -> None:
        B, H, D, W = self.batch, self.H, self.D, self.world
        scale = 1.0 if self.loss_reduction == "sum" else 1.0 / (B * W)
        p = self.params
        self._k.fwd_bwd(p["W1"], p["b1"], p["w2"], p["b2"], self.rows, self.dense, self.label, self.dense_row0, scale,
                        True, self.bufs, batch=B, step_ctr=self.step_ctr, feed=self.feed, rec_out=self.rec_idx)
        idx = self.rec_idx  # the records the kernel selected for this rank's rows of the global batch
        F = self.F
        sf = self.send[:4 * self.NF].view(torch.float32)
        seg = sf[:B * self.C].view(B, self.C)
        seg[:, :H] = self.bufs["a"]
        seg[:, H:2 * H] = self.bufs["dz"]
        seg[:, 2 * H:2 * H + D] = self.dense[idx]
        seg[:, 2 * H + D] = self.bufs["dlogit"]
        self.send[4 * self.NF:].view(torch.int32).view(B, F).copy_(self.rows[idx])
        if self.direct:
            sf[B * self.C:] = self.bufs["dpart"][:B * (D + 2) * H]
        self._all_gather()
        rv = self.recv.view(W, self.L)
        rf = rv[:, :4 * self.NF].contiguous().view(torch.float32)  # [W, NF]
        g = rf[:, :B * self.C].reshape(W * B, self.C)
        self.gbufs["a"].copy_(g[:, :H])
        self.gbufs["dz"].copy_(g[:, H:2 * H])
        self.g_xd.copy_(g[:, 2 * H:2 * H + D])
        self.gbufs["dlogit"].copy_(g[:, 2 * H + D])
        self.g_rows.copy_(rv[:, 4 * self.NF:].contiguous().view(torch.int32).view(W * B, F))
        if self.direct:
            self.gbufs["dpart"][:W * B * (D + 2) * H].view(W, -1).copy_(rf[:, B * self.C:])
        self._k.adagrad(p, self.accs, self.g_rows, self.g_xd, self.dense_row0, self.gbufs, self.lr, batch=W * B)
        self.step_ctr.add_(1)

    def set_data(self, ids: torch.Tensor, dense: torch.Tensor, label: torch.Tensor) -> None:
        """The training records (all of them, on every rank: each reads its slice of the global stream)."""
        self.rows = self.model.rows(ids.to(self.device)).to(torch.int32).contiguous()
        self.dense = dense.to(self.device).float().contiguous()
        self.label = label.to(self.device).float().contiguous()
        self.n = len(self.label)
        if self.n < self.batch:
            raise ValueError(f"{self.n} records < batch {self.batch}")
        if self.n < self.world * self.batch:
            raise ValueError(f"{self.n} records < one global batch ({self.world} x {self.batch})")
        if self.native:  # the device counter continues from the host's step count
            self.step_ctr.fill_(self.step_idx)
        # captured graphs hold the previous tensors' addresses and record count: recapture on the next step
        self.graph, self.graph_multi = None, None

    def _idx(self):
        from ..data.shuffle import record_indices

        gs, go, key = self.feed
        return torch.from_numpy(record_indices(self.step_idx, self.batch, self.n, gs, go, key)).to(self.device)

    def _native_step(self) -> None:
        if self.world > 1:
            self._native_step_dp()
            return
        scale = 1.0 if self.loss_reduction == "sum" else 1.0 / self.batch
        p = self.params
        self._k.fwd_bwd(p["W1"], p["b1"], p["w2"], p["b2"], self.rows, self.dense, self.label, self.dense_row0, scale,
                        True, self.bufs, batch=self.batch, step_ctr=self.step_ctr, feed=self.feed)
        self._k.adagrad(p, self.accs, self.rows, self.dense, self.dense_row0, self.bufs, self.lr, batch=self.batch,
                        step_ctr=self.step_ctr, feed=self.feed)

    def capture(self) -> None:
        """Capture one step and `steps_per_graph` consecutive steps as hipGraphs (every captured step reads the
        device counter, so replays walk through the data and the optimizer state like eager steps)."""
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._native_step()
        gm = None
        if self.steps_per_graph > 1:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm):
                for _ in range(self.steps_per_graph):
                    self._native_step()
        self.graph, self.graph_multi = g, gm

    def run(self, n: int) -> None:
        """n training steps: the first eagerly (lazy library/kernel initialisation), then multi-step graph replays
        and single-step replays for the remainder."""
        while n > 0 and self.use_graph and self.graph is None:
            self.step()  # step() captures once a first eager step has run
            n -= 1
        if self.graph_multi is not None:
            reps, n = divmod(n, self.steps_per_graph)
            for _ in range(reps):
                self.graph_multi.replay()
                self.step_idx += self.steps_per_graph
        for _ in range(n):
            self.step()

    def step(self) -> None:
        if self.native:
            if self.use_graph and self.graph is None and self.step_idx >= 1:  # first step eager (lazy init), then
                self.capture()
            if self.graph is not None:
                self.graph.replay()
            else:
                self._native_step()
            self._last_t = self.bufs["loss"]
        else:
            idx = self._idx()
            rows, xd, y = self.rows[idx].contiguous(), self.dense[idx].contiguous(), self.label[idx].contiguous()
            logit = self._forward_rows(rows, xd)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(logit, y, reduction=self.loss_reduction)
            self.opt.zero_grad(set_to_none=True)
            loss.backward()
            if self.world > 1:
                self.dp.finish()
            self.opt.step()
            self._last = float(loss.detach()) * (self.batch if self.loss_reduction == "mean" else 1.0)
        self.step_idx += 1

    def last_loss(self) -> float:
        if self.native:
            return float(self.bufs["loss"].sum())
        return self._last

    @torch.no_grad()
    def predict_logits(self, ids: torch.Tensor, dense: torch.Tensor, batch: int = 4096) -> np.ndarray:
        out = []
        for s in range(0, len(ids), batch):
            r = self.model.rows(ids[s:s + batch].to(self.device)).to(torch.int32).contiguous()
            xd = dense[s:s + batch].to(self.device).float().contiguous()
            if self.native:
                bufs = self._k.make_buffers(len(r), self.model.cfg.hidden, xd.shape[1], self.device)
                self._k.fwd_bwd(self.params["W1"], self.params["b1"], self.params["w2"], self.params["b2"], r, xd,
                                bufs["logit"], self.dense_row0, 1.0, False, bufs)
                out.append(bufs["logit"].cpu())
            else:
                out.append(self._forward_rows(r, xd).cpu())
        return torch.cat(out).numpy()

    def _forward_rows(self, rows: torch.Tensor, xd: torch.Tensor) -> torch.Tensor:
        """Reference forward on global W1 rows (what the HIP kernel computes)."""
        m = self.model
        z = m.b1 + m.W1[rows.long()].sum(1) + xd @ m.W1[self.dense_row0:]
        return torch.relu(z) @ m.w2 + m.b2
