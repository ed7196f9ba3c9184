"""AMD Instinct op modifiers: schedule an op onto MI355X nodes of a Kubernetes cluster.

No reference counterpart (the reference only knows `nvidia.com/gpu` and TPUs); this is the
MI355X-first equivalent of `gcp.use_tpu`. The AMD GPU device plugin exposes `amd.com/gpu`; the node
labeller publishes `amd.com/gpu.product-name` / `amd.com/gpu.family`. Multi-GPU ops get `/dev/shm`
sized for RCCL and `HSA_ENABLE_IPC_MODE_LEGACY=0` (dmabuf IPC, needed for RCCL peer access)."""
from __future__ import annotations

from .k8s import V1EmptyDirVolumeSource, V1EnvVar, V1Toleration, V1Volume, V1VolumeMount


def use_amd_gpus(num_gpus: int = 1, product: str | None = "MI355X", shm_size: str = "64Gi",
                 toleration: V1Toleration | None = None):
    """Request `num_gpus` AMD GPUs (one rank per GPU) with RCCL-friendly settings."""
    if num_gpus < 1:
        raise ValueError("num_gpus must be >= 1")

    def _use_amd_gpus(task):
        task.container.set_gpu_limit(str(num_gpus), vendor="amd")
        if product:
            task.add_node_selector_constraint("amd.com/gpu.product-name", product)
        if toleration is not None:
            task.add_toleration(toleration)
        task.container.add_env_variable(V1EnvVar(name="HSA_ENABLE_IPC_MODE_LEGACY", value="0"))
        task.container.add_env_variable(V1EnvVar(name="MIFX_NUM_GPUS", value=str(num_gpus)))
        if num_gpus > 1:
            task.add_volume(V1Volume(name="dshm", empty_dir=V1EmptyDirVolumeSource(medium="Memory",
                                                                                    size_limit=shm_size)))
            task.container.add_volume_mount(V1VolumeMount(name="dshm", mount_path="/dev/shm"))
        return task

    return _use_amd_gpus


def use_torchrun(num_gpus: int, master_port: int = 29500):
    """Wrap the op's command in a single-node `torch.distributed.run` launcher (one process per GPU)."""

    def _use_torchrun(task):
        c = task.container
        cmd = list(c.command or [])
        if cmd[:1] in (["python"], ["python3"]):
            cmd = cmd[1:]
        c.command = ["python3", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={num_gpus}",
                     "--master-addr=127.0.0.1", f"--master-port={master_port}"] + cmd
        return task

    return _use_torchrun
