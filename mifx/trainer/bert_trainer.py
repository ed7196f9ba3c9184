"""BERT fine-tune trainer (BASELINE config 4): tensor-parallel across the node's GPUs, bf16 autocast
with fp32 master weights, fused AdamW, synthetic GLUE-shaped batches (no dataset downloads).

`python -m torch.distributed.run --nproc-per-node 8 -m mifx.trainer.bert_trainer --steps 50` runs TP=8."""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

from ..models.bert import BertConfig, BertForSequenceClassification
from ..parallel import dist as mdist
from ..parallel.tensor_parallel import TPGroup
from ..utils.meter import heartbeat
from .optim import FlatAdamW


GEMM_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_bert_base_gfx950.csv")


def load_gemm_table(path: str = GEMM_TABLE) -> bool:
    """Use the hipBLASLt solutions recorded per BERT-base GEMM shape on an MI355X (PyTorch TunableOp results,
    read-only: no tuning at run time; shapes not in the table keep the library heuristic). Measured: 4592 ->
    4697 seq/s at B=32 S=128 (profiles/bert_base_bench_r2m*.json). Only on gfx950 with the table's library
    versions (TunableOp validates them and ignores a mismatching file)."""
    if not os.path.exists(path) or "gfx950" not in torch.cuda.get_device_properties(0).gcnArchName:
        return False
    import tempfile

    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(False)
    ok = bool(torch.cuda.tunable.read_file(path))
    # any results file TunableOp writes at exit goes to a scratch path, never over the bundled table
    torch.cuda.tunable.set_filename(os.path.join(tempfile.gettempdir(), f"mifx_tunableop_{os.getpid()}.csv"))
    return ok


def synthetic_batch(cfg: BertConfig, batch: int, seq: int, device, seed: int = 0):
    """Same tokens on every TP rank (TP ranks consume one replicated batch)."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(min(1000, cfg.vocab_size // 4), cfg.vocab_size, (batch, seq), generator=g)
    ids[:, 0] = 101  # [CLS]
    tt = torch.zeros(batch, seq, dtype=torch.long)
    tt[:, seq // 2:] = 1
    am = torch.ones(batch, seq)
    y = torch.randint(0, cfg.num_labels, (batch,), generator=g)
    return ids.to(device), tt.to(device), am.to(device), y.to(device)


class BertTrainer:
    """One fine-tuning step = forward + backward + fused AdamW. On the GPU the whole step (HIP LN/GELU /
    bias-grad kernels, hipBLASLt GEMMs, attention, dropout RNG, optimizer, and the TP all-reduces) is
    captured once into a hipGraph and replayed: the eager step is host-bound (12.8 ms wall for 10.0 ms of
    GPU work). The model weights are bf16 views of one flat buffer updated by a single fused HIP AdamW
    launch with fp32 master weights that reads autograd's own gradient tensors in place
    (mifx.trainer.optim.FlatAdamW): no per-step weight/grad cast kernels, no gradient zero-fill, no
    per-parameter accumulate kernels."""

    def __init__(self, cfg: BertConfig, batch: int, seq: int, device, tp: TPGroup | None = None, lr: float = 2e-5,
                 graph: bool | None = None, flat_adamw: bool | None = None, sdpa: str | None = None,
                 tp_ipc: bool | None = None):
        """tp_ipc (TP > 1 on the GPU; default on, MIFX_TP_IPC=0 turns it off): the TP all-reduces run on the
        peer-memory kernels of mifx.parallel.tp_ipc, so the TP step is captured into a hipGraph like the TP=1
        step (otherwise they are torch.distributed collectives and TP > 1 steps eagerly)."""
        self.cfg, self.batch, self.seq, self.device = cfg, batch, seq, torch.device(device)
        self.tp = tp or TPGroup(None)
        self.model = BertForSequenceClassification(cfg, self.tp, seed=0).to(self.device)
        cuda = self.device.type == "cuda"
        if tp_ipc is None:
            tp_ipc = os.environ.get("MIFX_TP_IPC", "1") != "0"
        if cuda and self.tp.size > 1 and tp_ipc:
            self.tp.enable_ipc(batch * seq * cfg.hidden, self.device)
        # The whole step is captured once as a hipGraph and replayed by default on the GPU (9.2 ms/step vs
        # 12.8 ms eager: the eager step is host-bound). The embeddings use a scatter-add backward
        # (mifx.ops.fused_bert.embedding): PyTorch's sort/unique embedding backward faults under hipGraph
        # replay on ROCm (rocPRIM partition kernel, diagnosed in round 1) and made the captured step go
        # non-finite after ~10 replays.
        # At TP > 1 the step is captured when the all-reduces are the peer-memory kernels (tp_ipc); over
        # torch.distributed collectives it steps eagerly unless graph=True is passed.
        self.use_graph = (cuda and (self.tp.size == 1 or self.tp.ipc is not None)) if graph is None \
            else (graph and cuda)
        self.flat = cuda if flat_adamw is None else (flat_adamw and cuda)
        if self.flat:  # bf16 weights/grads as flat-buffer views + fp32 master, one fused HIP update
            self.opt = FlatAdamW(self.model.parameters(), lr=lr, weight_decay=0.01)
        else:
            self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr, weight_decay=0.01, fused=cuda,
                                         capturable=self.use_graph)
        if self.model.sequence_parallel:
            if getattr(self.opt, "overlap", False):
                raise ValueError("sequence parallelism: the overlapped AdamW buckets would update the token-shard "
                                 "parameters before their gradients are summed over the group")
            if self.tp.ipc is not None and not self.tp.ipc.shard_ok(batch * seq * cfg.hidden):
                raise ValueError(f"sequence parallelism on the peer-memory path: batch x seq x hidden must split into "
                                 f"{self.tp.size} shards of whole {self.tp.ipc.chunk}-element chunks")
        # transposed copies of the projection weights for the dX GEMMs, refreshed in one launch before each backward
        self.tcache = None
        if self.flat:
            from ..ops import gemm as hg

            ws = [m.weight for layer in self.model.layers for m in (layer.qkv, layer.attn_out, layer.ffn_in,
                                                                      layer.ffn_out)]
            self.tcache = hg.TransposeCache(ws)
        self.data = synthetic_batch(cfg, batch, seq, self.device)
        self.amp = cuda
        self.sdpa = sdpa  # None = PyTorch's choice; "math" / "efficient" / "flash" pins the SDPA backend
        self.graph = None
        self.static_loss = None
        # MIFX_BERT_ASYNC_DW=1: weight gradients on a side stream (mifx.ops.gemm.async_weight_grads)
        self.async_dw = cuda and os.environ.get("MIFX_BERT_ASYNC_DW", "0") == "1"
        # deferred weight gradients (mifx.ops.gemm.deferred_weight_grads; MIFX_DEFER_DW=0 turns it off): the flat
        # optimizer resets every gradient to None each step, which the flush relies on
        self.defer_dw = cuda and self.flat and not self.async_dw and os.environ.get("MIFX_DEFER_DW", "1") != "0"
        # (TP ranks sharing one device -- the one-GPU rehearsals -- used to need it off: the grouped launch's
        # workgroups need a whole CU's register file, which the other ranks' spinning all-reduce waves held. The IPC
        # all-reduce now switches itself to split waits when ranks share a device (mifx.parallel.tp_ipc: no
        # data-moving workgroup spins, one wave waits), so the flush always finds whole CUs and the rehearsed step is
        # the shipped one.)

    def set_batch(self, ids, tt, am, y) -> None:
        """Next training batch, copied INTO the step's input tensors (a captured hipGraph reads these same
        buffers on every replay)."""
        for dst, src in zip(self.data, (ids, tt, am, y)):
            dst.copy_(src.to(dst.dtype), non_blocking=True)

    @torch.no_grad()
    def predict(self, ids, tt, am) -> torch.Tensor:
        """Eval-mode logits (every TP rank must call it: the forward all-reduces)."""
        self.model.eval()
        try:
            with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
                return self.model(ids.to(self.device), tt.to(self.device), am.to(self.device).float()).float()
        finally:
            self.model.train()

    def _eager_step(self) -> torch.Tensor:
        ids, tt, am, y = self.data
        if self.flat:
            self.opt.zero_grad()  # in-place (gradients are views of one flat buffer): part of the step
        # the autocast weight-cast cache must be off for a step that is captured into a graph (PyTorch's
        # CUDA-graph rules: cached casts created outside the capture must not be referenced by it)
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp,
                            cache_enabled=not self.use_graph), self._sdpa_ctx():
            logits = self.model(ids, tt, am)
        loss = F.cross_entropy(logits.float(), y)
        from ..ops import gemm as hg

        if self.tcache is not None:
            # the transposed weight copies the dX GEMMs read, refreshed from the CURRENT weights right before the
            # backward (once per step, inside the captured graph): a weight change between steps (an update, a
            # load_state_dict, a warm start) can never leave the backward with stale transposes
            self.tcache.refresh()
        with hg.use_transposes(self.tcache):
            if self.async_dw:  # weight-gradient GEMMs on a side stream beside the backward's dX chain
                with hg.async_weight_grads():
                    loss.backward()
                hg.join_weight_grads(self.device)
            elif self.defer_dw:  # every weight gradient in ONE grouped launch after the backward
                with hg.deferred_weight_grads():
                    loss.backward()
                hg.flush_weight_grads()
            else:
                loss.backward()
        # sequence parallelism: the LayerNorm / row-parallel-bias gradients are per-shard partial sums
        self.model.sync_sequence_parallel_grads()
        self.opt.step()
        return loss.detach()

    def _sdpa_ctx(self):
        if self.sdpa is None:
            return contextlib.nullcontext()
        from torch.nn.attention import SDPBackend, sdpa_kernel

        return sdpa_kernel({"math": SDPBackend.MATH, "efficient": SDPBackend.EFFICIENT_ATTENTION,
                            "flash": SDPBackend.FLASH_ATTENTION}[self.sdpa])

    def _capture(self, warmup: int = 3) -> None:
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):  # warm up on a side stream: lazy state (AdamW moments, caches)
            for _ in range(warmup):
                self.opt.zero_grad(set_to_none=True)
                self._eager_step()
        torch.cuda.current_stream(self.device).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        self.opt.zero_grad(set_to_none=True)
        if hasattr(self.opt, "begin_capture"):  # FlatAdamW: bucket updates overlapped with the backward
            self.opt.begin_capture()
        with torch.cuda.graph(self.graph):
            self.static_loss = self._eager_step()

    # TP health check cadence: the peer-memory all-reduce reports a peer that never arrived through a sticky device
    # flag (its later kernels then write NaN); reading it is a host sync, so step() reads it every CHECK_EVERY steps
    CHECK_EVERY = 100

    def check(self) -> None:
        """Raise if a TP all-reduce of this trainer's group timed out (no-op at TP = 1 / without the IPC path)."""
        self.tp.check()

    def step(self) -> torch.Tensor:
        self.steps_done = getattr(self, "steps_done", 0) + 1
        if self.tp.ipc is not None and self.steps_done % self.CHECK_EVERY == 0:
            self.check()
        if self.use_graph:
            if self.graph is None:
                self._capture()
            self.graph.replay()
            return self.static_loss
        self.opt.zero_grad(set_to_none=True)
        return self._eager_step()

    def load_weights(self, state: dict) -> None:
        """Load a (full or TP-sharded) state dict into the model and refresh everything derived from the weights
        (the transposed copies of the dX GEMMs). Use this instead of model.load_state_dict after construction."""
        self.model.load_state_dict(state)
        if self.flat and hasattr(self.opt, "reload_master"):
            self.opt.reload_master()
        if self.tcache is not None:
            self.tcache.refresh()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--graph", action="store_true", help="capture the step as one hipGraph also at TP>1")
    ap.add_argument("--no-graph", action="store_true", help="eager steps instead of one captured hipGraph")
    ap.add_argument("--no-flat-adamw", action="store_true",
                    help="eager mode: fp32 params + torch fused AdamW instead of the flat HIP AdamW")
    ap.add_argument("--tunable", default=None, metavar="CSV",
                    help="enable PyTorch TunableOp: benchmark hipBLASLt/rocBLAS solutions per GEMM shape during "
                         "warmup and keep the best (results cached in CSV)")
    ap.add_argument("--no-gemm-table", action="store_true",
                    help="do not load the bundled per-shape GEMM solution table (tunableop_bert_base_gfx950.csv)")
    ap.add_argument("--seed", type=int, default=None, help="torch.manual_seed before building the trainer")
    ap.add_argument("--dropout", type=float, default=0.1)
    ap.add_argument("--sequence-parallel", action="store_true",
                    help="at TP > 1: split the residual stream / LayerNorms / dropouts over the ranks by token")
    ap.add_argument("--sdpa", choices=["math", "efficient", "flash"], default=None,
                    help="pin the scaled-dot-product-attention backend (default: PyTorch's choice)")
    a = ap.parse_args(argv)
    if a.seed is not None:
        torch.manual_seed(a.seed)
    if a.tunable and torch.cuda.is_available():
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(a.tunable)
        torch.cuda.tunable.set_max_tuning_iterations(30)
    elif not a.no_gemm_table and os.environ.get("MIFX_BERT_GEMM_TABLE", "1") != "0" and torch.cuda.is_available():
        load_gemm_table()
    env = mdist.init()
    # MIFX_SHARED_GPU=1 (with MIFX_DIST_BACKEND=gloo): the multi-rank flow rehearsed with every rank on cuda:0
    local = 0 if os.environ.get("MIFX_SHARED_GPU") == "1" else env.local_rank
    dev = torch.device("cuda", local) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    tp = TPGroup(torch.distributed.group.WORLD if env.world_size > 1 else None)
    cfg = BertConfig(layers=a.layers, dropout=a.dropout, sequence_parallel=a.sequence_parallel)
    tr = BertTrainer(cfg, a.batch, a.seq, dev, tp,
                     graph=False if a.no_graph else (True if a.graph else None),
                     flat_adamw=False if a.no_flat_adamw else None, sdpa=a.sdpa)
    from ..ops import native_stats

    per_step = None
    with heartbeat("bert warmup"):
        for i in range(a.warmup):
            if i == 0:
                native_stats.reset()
            tr.step()
            if i == 0:  # the first step runs every dispatch in Python: which path each GEMM / attention call took
                per_step = native_stats.snapshot()
        if dev.type == "cuda":
            torch.cuda.synchronize()
    tr.check()  # a timed-out TP all-reduce during warmup fails the run here (outside the timed region)
    mdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    trace = os.environ.get("MIFX_BERT_TRACE") == "1"  # diagnostic: per-step loss (adds a sync per step)
    sync_each = os.environ.get("MIFX_BERT_SYNC") == "1"  # diagnostic: device sync after every step
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = tr.step()
        if sync_each and dev.type == "cuda":
            torch.cuda.synchronize()
        if trace and env.rank == 0:
            print(f"[bert] step {i} loss {float(loss):.5f}", file=sys.stderr, flush=True)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    mdist.barrier()
    dt = mdist.max_over_ranks(time.perf_counter() - t0)
    tr.check()  # ... and during the timed steps: never report a throughput of garbage activations
    if env.rank == 0:
        print(json.dumps({"metric": "BERT-base fine-tune sequences/sec (TP over the node)", "value": a.batch * a.steps / dt,
                          "unit": "sequences/s", "n_gpus": env.world_size, "tp": tp.size,
                          "sequence_parallel": tr.model.sequence_parallel, "batch": a.batch,
                          "seq_len": a.seq, "ms_per_step": 1e3 * dt / a.steps, "loss": float(loss),
                          "dtype": "bf16", "data": "synthetic", "layers": a.layers,
                          "hipgraph": tr.graph is not None,
                          "calls_per_step_native_vs_fallback": per_step,
                          "optimizer": "flat bf16 AdamW (fp32 master)" if tr.flat else "torch fused AdamW"}),
              flush=True)
    mdist.shutdown()


if __name__ == "__main__":
    main()
