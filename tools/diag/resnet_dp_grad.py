"""Diagnostic: ResNet-50 DP=2 on one GPU (gloo) -- compare each rank's local gradient (no_sync) with the
DP-averaged gradient of the same batch, and the two ranks' local gradients with each other."""
import os
import socket
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mifx.ops.image_ops import crop_flip_normalize
    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    imgs, labels = synthetic_imagenet(64, size=72, classes=10, seed=0)
    tr = ResNetTrainer(4, "cuda:0", imgs, labels, num_classes=10, lr=0.002, warmup_steps=1, crop=64,
                       process_group=dist.group.WORLD, seed=3)
    torch.backends.cudnn.benchmark = False
    idx = torch.arange(4, device="cuda:0")
    x = crop_flip_normalize(tr.images, idx, (64, 64), False, 0, 0, tr.mean, tr.std, torch.bfloat16)
    y = tr.labels[idx]
    params = [p for p in tr.model.parameters()]

    def grads(sync):
        for p in params:
            p.grad = None
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(tr.model(x).float(), y)
        if sync:
            loss.backward()
            tr.dp.finish()
        else:
            with tr.dp.no_sync():
                loss.backward()
        torch.cuda.synchronize()
        return float(loss), [p.grad.detach().float().cpu().clone() for p in params]

    l0, g_local = grads(False)
    l0b, g_local2 = grads(False)
    l1, g_dp = grads(True)
    torch.save({"loss": (l0, l0b, l1), "local": g_local, "local2": g_local2, "dp": g_dp}, f"{out}.{rank}")
    dist.destroy_process_group()


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


if __name__ == "__main__":
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "g")
        mp.start_processes(worker, args=(2, port, out), nprocs=2, start_method="spawn")
        r = [torch.load(f"{out}.{i}", weights_only=True) for i in range(2)]
    print("losses", r[0]["loss"], r[1]["loss"])
    worst = {}
    for name, a, b in (("local vs local2 (same proc)", r[0]["local"], r[0]["local2"]),
                       ("rank0 local vs rank1 local", r[0]["local"], r[1]["local"]),
                       ("rank0 dp vs rank0 local", r[0]["dp"], r[0]["local"]),
                       ("rank0 dp vs mean(local0, local1)", r[0]["dp"], [(u + v) / 2 for u, v in zip(r[0]["local"], r[1]["local"])]),
                       ("rank0 dp vs rank1 dp", r[0]["dp"], r[1]["dp"])):
        vals = [rel(u, v) for u, v in zip(a, b)]
        print(f"{name:40s} max rel {max(vals):.3e}  median {sorted(vals)[len(vals)//2]:.3e}  argmax {vals.index(max(vals))}")
