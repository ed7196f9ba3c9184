"""Diagnostics for the xGMI exchange (mifx.parallel.xgmi) with W processes sharing one GPU:
1. raw exchange stress: N epochs of (rank, epoch)-dependent patterns through sum_into, exact compare;
2. W&D DP step-by-step (eager) against one process stepping on the global batch: max |diff| per step.
usage: python tools/xgmi_probe.py [--world 2] [--iters 200] [--steps 6]"""
import argparse
import os
import socket
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, iters, steps, batch):
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.parallel.xgmi import XgmiExchange
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    stride = 20608
    xg = XgmiExchange(stride, dist.group.WORLD, dev)
    xg.selftest()
    i = torch.arange(stride, device=dev, dtype=torch.float32)
    bad, first = 0, None
    out = torch.empty(stride, device=dev)
    for it in range(iters):
        base = torch.remainder(i + it, 89) + 1
        mine = ((rank + 1) * base).view(1, -1)
        want = (world * (world + 1) // 2) * base
        xg.sum_into(mine, out)
        if it % 7 == 0:
            torch.cuda.synchronize()  # mix lock-step and free-running epochs
        if not torch.equal(out, want):
            bad += 1
            first = it if first is None else first
    xg.check()
    print(f"[rank {rank}] exchange stress: {iters} epochs, {bad} wrong (first {first})", flush=True)
    xg.close()

    recs = synthetic_records(batch * world * steps, device="cpu", seed=11)
    shard = recs.view(steps, world, batch, 32)[:, rank].reshape(-1, 32).contiguous()
    tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device=dev, process_group=dist.group.WORLD)
    tr.set_data(shard.cuda())
    tr.enable_xgmi()
    ref = None
    if rank == 0:
        ref = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch * world, device=dev)
        ref.set_data(recs.cuda())
    for st in range(steps):
        tr.step()
        torch.cuda.synchronize()
        if rank == 0:
            ref.step()
            torch.cuda.synchronize()
            d = (tr.param - ref.param).abs()
            print(f"[step {st}] max|diff| {d.max().item():.3e}  dnn {d[:wdm.WTOT].max().item():.3e}  "
                  f"wide {d[wdm.WTOT:].max().item():.3e}  step_ctr {tr.steps_done}/{ref.steps_done}  "
                  f"xctr {int(tr._xg.xctr[0].item())}", flush=True)
        dist.barrier()
    tr._xg.check()
    tr.disable_xgmi()

    # 3. free-running ranks (no per-step sync): eager, then graphs, then first step on the collective path
    split = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device=dev, process_group=dist.group.WORLD)
    split.set_data(shard.cuda())
    split.capture(dp_mode="split")
    split.run(steps - 2)
    torch.cuda.synchronize()
    split_param = split.param.clone()
    for mode in ("eager-free", "graph", "collective-first+graph"):
        tr = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch, device=dev, process_group=dist.group.WORLD)
        tr.set_data(shard.cuda())
        n = steps
        if mode == "collective-first+graph":
            tr.step()
            n -= 1
        if mode == "eager-free":
            tr.enable_xgmi()
            for _ in range(n):
                tr.step()
        else:
            tr.capture(warmup=1, steps_per_graph=3, dp_mode="xgmi")
            tr.run(n - 1)
        torch.cuda.synchronize()
        tr._xg.check()
        if rank == 0:
            ref = FusedWideDeepTrainer(wdm.WideDeepModel(seed=5), batch=batch * world, device=dev)
            ref.set_data(recs.cuda())
            for _ in range(steps):
                ref.step()
            torch.cuda.synchronize()
            d = (tr.param - ref.param).abs()
            ds = (tr.param - split_param).abs().max().item()
            dr = (split_param - ref.param).abs().max().item()
            print(f"[{mode}] {steps} steps: max|xgmi - single| {d.max().item():.3e}  max|xgmi - split-phase DP| "
                  f"{ds:.3e}  max|split-phase DP - single| {dr:.3e}  step_ctr {tr.steps_done}/{ref.steps_done}",
                  flush=True)
        tr.disable_xgmi()
    dist.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    mp.start_processes(worker, args=(a.world, _port(), a.iters, a.steps, a.batch), nprocs=a.world,
                       start_method="spawn")
