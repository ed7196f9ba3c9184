"""Diagnostic: ResNet-50 trainer, 2 ranks sharing cuda:0 (gloo group), bucket exchange "ipc" vs "rccl" (the group's
collective) vs one process accumulating both micro-batches: per-step losses of every rank, and where the first
parameter difference between the two exchanges appears. Prints one JSON line."""
import json
import os
import socket
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

STEPS = int(os.environ.get("DIAG_STEPS", "3"))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, out, exchange, graph):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), MIFX_DP_EXCHANGE=exchange)
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    imgs, labels = synthetic_imagenet(64, size=72, classes=10, seed=0)
    tr = ResNetTrainer(4, "cuda:0", imgs, labels, num_classes=10, lr=0.05, warmup_steps=1, crop=64,
                       process_group=dist.group.WORLD if world > 1 else None, seed=3,
                       accum_steps=1 if world > 1 else 2, graph=graph)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    losses, sums = [], []
    for _ in range(STEPS):
        losses.append(float(tr.step()))
        torch.cuda.synchronize()
        sums.append({k: float(v.detach().double().sum()) for k, v in tr.model.named_parameters()})
    torch.save({"losses": losses, "sums": sums}, f"{out}.{exchange}.{graph}.{world}.{rank}")
    if world > 1:
        dist.destroy_process_group()


def main():
    res = {}
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r")
        for exchange in ("ipc", "rccl"):
            for graph in (False, True):
                mp.start_processes(worker, args=(2, _port(), out, exchange, graph), nprocs=2, start_method="spawn")
                res[(exchange, graph)] = [torch.load(f"{out}.{exchange}.{graph}.2.{r}", weights_only=True)
                                          for r in range(2)]
        mp.start_processes(worker, args=(1, _port(), out, "rccl", False), nprocs=1, start_method="spawn")
        one = torch.load(f"{out}.rccl.False.1.0", weights_only=True)
    rep = {"single": one["losses"]}
    for (exchange, graph), rr in res.items():
        rep[f"{exchange}_graph{int(graph)}"] = [r["losses"] for r in rr]
    # first step / parameter where ipc and rccl (eager) differ
    a, b = res[("ipc", False)][0]["sums"], res[("rccl", False)][0]["sums"]
    diffs = []
    for s in range(STEPS):
        for k in a[s]:
            if a[s][k] != b[s][k]:
                diffs.append((s, k, a[s][k], b[s][k]))
    rep["first_ipc_rccl_param_diffs"] = diffs[:8]
    print(json.dumps(rep), flush=True)


if __name__ == "__main__":
    main()
