"""Process-group helpers: one process per GPU, RCCL ("nccl" backend on ROCm) over xGMI, or gloo
on CPU. Replaces the reference's TFJob/MPIJob/PyTorchJob operators for single-node DP
(`notebooks/training-jobs/distributed-tensorflow-training-job.yaml:1-18`)."""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistEnv:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_from_os() -> DistEnv:
    return DistEnv(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                   int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str | None = None, timeout_s: int = 600) -> DistEnv:
    """Initialise torch.distributed from torchrun-style env vars (no-op when WORLD_SIZE == 1)."""
    env = env_from_os()
    if env.world_size == 1:
        return env
    if dist.is_initialized():
        env.backend = dist.get_backend()
        return env
    if backend is None:  # MIFX_DIST_BACKEND: rehearsal override (e.g. gloo ranks sharing one GPU)
        backend = os.environ.get("MIFX_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if backend == "nccl":
        torch.cuda.set_device(env.local_rank)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s),
                                device_id=torch.device("cuda", env.local_rank))
    else:
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=timeout_s))
    env.backend = backend
    return env


def barrier() -> None:
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def max_over_ranks(x: float, device=None) -> float:
    if not dist.is_initialized():
        return x
    if device is None and dist.get_backend() == "nccl":  # RCCL reduces device tensors only
        device = torch.device("cuda", torch.cuda.current_device())
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
