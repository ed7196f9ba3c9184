"""BERT fine-tune trainer (BASELINE config 4): tensor-parallel across the node's GPUs, bf16 autocast
with fp32 master weights, fused AdamW, synthetic GLUE-shaped batches (no dataset downloads).

`python -m torch.distributed.run --nproc-per-node 8 -m mifx.trainer.bert_trainer --steps 50` runs TP=8."""
from __future__ import annotations

import argparse
import json
import os
import time

import torch
import torch.nn.functional as F

from ..models.bert import BertConfig, BertForSequenceClassification
from ..parallel import dist as mdist
from ..parallel.tensor_parallel import TPGroup


def synthetic_batch(cfg: BertConfig, batch: int, seq: int, device, seed: int = 0):
    """Same tokens on every TP rank (TP ranks consume one replicated batch)."""
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(1000, cfg.vocab_size, (batch, seq), generator=g)
    ids[:, 0] = 101  # [CLS]
    tt = torch.zeros(batch, seq, dtype=torch.long)
    tt[:, seq // 2:] = 1
    am = torch.ones(batch, seq)
    y = torch.randint(0, cfg.num_labels, (batch,), generator=g)
    return ids.to(device), tt.to(device), am.to(device), y.to(device)


class BertTrainer:
    def __init__(self, cfg: BertConfig, batch: int, seq: int, device, tp: TPGroup | None = None, lr: float = 2e-5):
        self.cfg, self.batch, self.seq, self.device = cfg, batch, seq, torch.device(device)
        self.tp = tp or TPGroup(None)
        self.model = BertForSequenceClassification(cfg, self.tp, seed=0).to(self.device)
        fused = self.device.type == "cuda"
        self.opt = torch.optim.AdamW(self.model.parameters(), lr=lr, weight_decay=0.01, fused=fused)
        self.data = synthetic_batch(cfg, batch, seq, self.device)
        self.amp = self.device.type == "cuda"

    def step(self) -> torch.Tensor:
        ids, tt, am, y = self.data
        self.opt.zero_grad(set_to_none=True)
        with torch.autocast(self.device.type, dtype=torch.bfloat16, enabled=self.amp):
            logits = self.model(ids, tt, am)
        loss = F.cross_entropy(logits.float(), y)
        loss.backward()
        self.opt.step()
        return loss.detach()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--seq", type=int, default=128)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--layers", type=int, default=12)
    a = ap.parse_args(argv)
    env = mdist.init()
    dev = torch.device("cuda", env.local_rank) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    tp = TPGroup(torch.distributed.group.WORLD if env.world_size > 1 else None)
    tr = BertTrainer(BertConfig(layers=a.layers), a.batch, a.seq, dev, tp)
    for _ in range(a.warmup):
        tr.step()
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
    if env.rank == 0:
        print(json.dumps({"metric": "BERT-base fine-tune sequences/sec (TP over the node)", "value": a.batch * a.steps / dt,
                          "unit": "sequences/s", "n_gpus": env.world_size, "tp": tp.size, "batch": a.batch,
                          "seq_len": a.seq, "ms_per_step": 1e3 * dt / a.steps, "loss": float(loss),
                          "dtype": "bf16", "data": "synthetic", "layers": a.layers}), flush=True)
    mdist.shutdown()


if __name__ == "__main__":
    main()
