"""Probe: can two ranks share ONE GPU over RCCL on this box (so a multi-rank captured-collective step can be
exercised without a multi-GPU node)? Each rank all-reduces a tensor eagerly and inside a hipGraph."""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=2, device_id=torch.device("cuda", 0))
    x = torch.full((1024,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print(f"rank {rank} eager all_reduce -> {x[0].item()}", flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dist.all_reduce(x)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    y = torch.full((1024,), float(rank + 1), device="cuda")
    with torch.cuda.graph(g):
        dist.all_reduce(y)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    print(f"rank {rank} graph all_reduce x3 -> {y[0].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    mp.start_processes(worker, args=(int(sys.argv[1]) if len(sys.argv) > 1 else 29533,), nprocs=2, start_method="spawn")
