from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time
from dataclasses import dataclass, field

import yaml

_SPEC_KEYS = {"TFJob": "tfReplicaSpecs", "PyTorchJob": "pytorchReplicaSpecs", "MPIJob": "mpiReplicaSpecs",
              "MIFXJob": "replicaSpecs"}
_ORDER = ("Chief", "Master", "Launcher", "Worker", "PS", "Evaluator")


@dataclass
class ReplicaSpec:
    role: str
    replicas: int
    command: list
    env: dict = field(default_factory=dict)
    gpus: int = 0
    image: str = ""
    restart_policy: str = "Never"


@dataclass
class JobSpec:
    kind: str
    name: str
    replicas: list  # [ReplicaSpec] in launch order

    @property
    def world_size(self) -> int:
        return sum(r.replicas for r in self.replicas if r.role != "PS")

    @staticmethod
    def from_dict(d: dict) -> "JobSpec":
        kind = d.get("kind", "MIFXJob")
        key = _SPEC_KEYS.get(kind)
        if key is None:
            raise ValueError(f"unsupported job kind {kind}")
        specs = d.get("spec", {}).get(key, {})
        out = []
        for role in sorted(specs, key=lambda r: _ORDER.index(r) if r in _ORDER else 99):
            s = specs[role]
            c = s.get("template", {}).get("spec", {}).get("containers", [{}])[0]
            lim = (c.get("resources") or {}).get("limits") or {}
            gpus = int(lim.get("amd.com/gpu", lim.get("nvidia.com/gpu", 0)) or 0)
            env = {e["name"]: str(e.get("value", "")) for e in c.get("env", []) or []}
            out.append(ReplicaSpec(role, int(s.get("replicas", 1)), list(c.get("command", [])) + list(c.get("args", [])),
                                   env, gpus, c.get("image", ""), s.get("restartPolicy", "Never")))
        spec = JobSpec(kind, d.get("metadata", {}).get("name", "job"), out)
        validate(spec)
        return spec

    @staticmethod
    def from_yaml(path: str) -> "JobSpec":
        with open(path) as f:
            return JobSpec.from_dict(yaml.safe_load(f))


def validate(spec: JobSpec) -> None:
    """CRD-equivalent validation (TFJob: Worker/PS/Chief replicas >= 1, Chief <= 1; Master <= 1)."""
    for r in spec.replicas:
        if r.replicas < 1:
            raise ValueError(f"{r.role}.replicas must be >= 1")
        if r.role in ("Chief", "Master", "Launcher") and r.replicas > 1:
            raise ValueError(f"{r.role}.replicas must be <= 1")
        if not r.command:
            raise ValueError(f"{r.role}: container command is required")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tf_config(spec: JobSpec, role: str, index: int, base_port: int) -> str:
    cluster, port = {}, base_port
    for r in spec.replicas:
        cluster[r.role.lower()] = [f"127.0.0.1:{port + i}" for i in range(r.replicas)]
        port += r.replicas
    return json.dumps({"cluster": cluster, "task": {"type": role.lower(), "index": index}, "environment": "cloud"})


def launch_local(spec: JobSpec, num_gpus: int | None = None, timeout: float | None = None, cwd: str | None = None,
                 log_dir: str | None = None) -> dict:
    """Run every replica as a local process; returns {role-index: exit code} (and logs under log_dir)."""
    if num_gpus is None:
        try:
            import torch

            num_gpus = torch.cuda.device_count()
        except Exception:  # noqa: BLE001
            num_gpus = 0
    port = _free_port()
    tf_port = _free_port()
    procs, rank = {}, 0
    log_dir = log_dir or os.path.join("/tmp", f"mifx_job_{spec.name}")
    os.makedirs(log_dir, exist_ok=True)
    for r in spec.replicas:
        for i in range(r.replicas):
            env = dict(os.environ, **r.env)
            is_rank = r.role != "PS"
            env.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(spec.world_size),
                        "HSA_ENABLE_IPC_MODE_LEGACY": "0", "JOB_ROLE": r.role, "JOB_INDEX": str(i)})
            if is_rank:
                env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(spec.world_size)})
                if num_gpus:
                    env["HIP_VISIBLE_DEVICES"] = str(rank % num_gpus)
                    env["LOCAL_RANK"] = "0"  # one visible device per process
            if spec.kind == "TFJob":
                env["TF_CONFIG"] = _tf_config(spec, r.role, i, tf_port)
            cmd = [sys.executable if c in ("python", "python3") else c for c in r.command]
            log = open(os.path.join(log_dir, f"{r.role.lower()}-{i}.log"), "w")
            procs[f"{r.role.lower()}-{i}"] = (subprocess.Popen(cmd, env=env, cwd=cwd, stdout=log,
                                                               stderr=subprocess.STDOUT), log)
            if is_rank:
                rank += 1
    deadline = time.time() + timeout if timeout else None
    codes = {}
    for k, (p, log) in procs.items():
        try:
            codes[k] = p.wait(timeout=max(1.0, deadline - time.time()) if deadline else None)
        except subprocess.TimeoutExpired:
            p.kill()
            codes[k] = -9
        log.close()
    if any(c != 0 for c in codes.values()):  # a failed rank takes the job down (restartPolicy Never)
        for p, _ in procs.values():
            if p.poll() is None:
                p.kill()
    return codes


def to_indexed_job(spec: JobSpec, namespace: str = "kubeflow", image: str | None = None) -> dict:
    """Single-node k8s Job that runs the ranks with torch.distributed.run inside one pod (all GPUs of a node)."""
    workers = [r for r in spec.replicas if r.role != "PS"]
    n = sum(r.replicas for r in workers)
    gpus = sum(r.gpus * r.replicas for r in workers) or n
    cmd = workers[0].command
    if cmd[:1] in (["python"], ["python3"]):
        cmd = cmd[1:]
    container = {"name": spec.name, "image": image or workers[0].image or "mifx/mifx-rocm:latest",
                 "command": ["python3", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
                             "--master-addr=127.0.0.1"] + cmd,
                 "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}],
                 "resources": {"limits": {"amd.com/gpu": str(gpus)}},
                 "volumeMounts": [{"name": "dshm", "mountPath": "/dev/shm"}]}
    return {"apiVersion": "batch/v1", "kind": "Job", "metadata": {"name": spec.name, "namespace": namespace},
            "spec": {"backoffLimit": 0, "template": {"spec": {
                "restartPolicy": "Never", "containers": [container],
                "volumes": [{"name": "dshm", "emptyDir": {"medium": "Memory", "sizeLimit": "64Gi"}}]}}}}


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(prog="python -m mifx.launch.job")
    ap.add_argument("spec")
    ap.add_argument("--render", action="store_true", help="print the k8s Job instead of running locally")
    ap.add_argument("--timeout", type=float, default=None)
    a = ap.parse_args(argv)
    spec = JobSpec.from_yaml(a.spec)
    if a.render:
        print(yaml.safe_dump(to_indexed_job(spec), sort_keys=False))
        return 0
    codes = launch_local(spec, timeout=a.timeout)
    print(json.dumps(codes))
    return 0 if all(c == 0 for c in codes.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
