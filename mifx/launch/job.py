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
    backoff_limit: int | None = None  # spec.runPolicy.backoffLimit (kubeflow v1) / spec.backoffLimit

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
        sp = d.get("spec", {}) or {}
        bl = (sp.get("runPolicy") or {}).get("backoffLimit", sp.get("backoffLimit"))
        spec = JobSpec(kind, d.get("metadata", {}).get("name", "job"), out, None if bl is None else int(bl))
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
        if r.restart_policy not in ("Never", "OnFailure", "Always", "ExitCode"):
            raise ValueError(f"{r.role}.restartPolicy must be one of Never, OnFailure, Always, ExitCode")
    if spec.backoff_limit is not None and spec.backoff_limit < 0:
        raise ValueError("backoffLimit must be >= 0")


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


# Exit codes the "ExitCode" restart policy treats as retryable (Kubeflow training-operator semantics: 128 + signal,
# e.g. 137 OOM-kill / SIGKILL, 143 SIGTERM, 130 SIGINT; 1-127 are the program's own, permanent, failures)
def _retryable(code: int) -> bool:
    return code < 0 or code >= 128


def _wants_restart(spec: JobSpec, codes: dict, roles: dict) -> bool:
    """Does the failed replica set restart? Only when EVERY failing replica's policy allows it (a permanent failure of
    any one replica ends the job)."""
    failed = [(k, c) for k, c in codes.items() if c != 0]
    if not failed:
        return False
    for k, c in failed:
        pol = roles[k].restart_policy
        if pol in ("OnFailure", "Always"):
            continue
        if pol == "ExitCode" and _retryable(c):
            continue
        return False
    return True


def launch_local(spec: JobSpec, num_gpus: int | None = None, timeout: float | None = None, cwd: str | None = None,
                 log_dir: str | None = None, isolate_gpus: bool = False, backoff_limit: int | None = None,
                 backoff_s: float = 0.5, stats: dict | None = None) -> dict:
    """Run every replica as a local process; returns {role-index: exit code} of the last attempt (logs under log_dir).

    GPUs: every rank sees ALL of the node's GPUs and gets LOCAL_RANK = its rank on the node (torchrun's contract), so
    a data-parallel job can map its peers' HBM over xGMI (IPC gradient exchange) and RCCL can use P2P; only
    `isolate_gpus=True` (independent processes such as HPO trials) pins one device per process through
    HIP_VISIBLE_DEVICES.

    Failures: the first replica that exits non-zero takes the whole replica set down (torch.distributed ranks cannot
    rejoin a group one at a time). With `restartPolicy: Never` (the reference's TFJob default) that ends the job. With
    `OnFailure` / `Always` (or `ExitCode` and a retryable code >= 128) the whole set is relaunched as FRESH processes --
    MIFX_RESTART_COUNT = the attempt number, same ports, same ranks -- after a bounded exponential backoff, at most
    `backoff_limit` times (default: the spec's runPolicy.backoffLimit, else 3); the workload resumes from its latest
    checkpoint (the estimator / Trainer components do that on start). `stats` (if given) receives {"restarts": n,
    "attempts": [codes of every attempt]}."""
    if num_gpus is None:
        try:
            import torch

            num_gpus = torch.cuda.device_count()
        except Exception:  # noqa: BLE001
            num_gpus = 0
    if backoff_limit is None:
        backoff_limit = spec.backoff_limit if spec.backoff_limit is not None else 3
    log_dir = log_dir or os.path.join("/tmp", f"mifx_job_{spec.name}")
    os.makedirs(log_dir, exist_ok=True)
    deadline = time.time() + timeout if timeout else None
    attempts = []
    attempt = 0
    while True:
        codes, roles = _run_once(spec, num_gpus, deadline, cwd, log_dir, isolate_gpus, attempt)
        attempts.append(codes)
        timed_out = any(c == -9 for c in codes.values()) and deadline is not None and time.time() >= deadline
        if timed_out or attempt >= backoff_limit or not _wants_restart(spec, codes, roles):
            break
        attempt += 1
        time.sleep(min(backoff_s * 2 ** (attempt - 1), 30.0))
    if stats is not None:
        stats["restarts"] = attempt
        stats["attempts"] = attempts
    return codes


def _run_once(spec: JobSpec, num_gpus: int, deadline, cwd, log_dir, isolate_gpus: bool, attempt: int):
    port = _free_port()
    tf_port = _free_port()
    procs, roles, rank = {}, {}, 0
    for r in spec.replicas:
        for i in range(r.replicas):
            env = dict(os.environ, **r.env)
            is_rank = r.role != "PS"
            env.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "WORLD_SIZE": str(spec.world_size),
                        "HSA_ENABLE_IPC_MODE_LEGACY": "0", "JOB_ROLE": r.role, "JOB_INDEX": str(i),
                        "MIFX_RESTART_COUNT": str(attempt)})
            if is_rank:
                env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(spec.world_size)})
                if num_gpus:
                    if isolate_gpus:
                        env["HIP_VISIBLE_DEVICES"] = str(rank % num_gpus)
                        env["LOCAL_RANK"] = "0"  # one visible device per process
                    else:  # (visibility left as inherited, like torchrun: every device, peers reachable over xGMI)
                        env["LOCAL_RANK"] = str(rank % num_gpus)
            if spec.kind == "TFJob":
                env["TF_CONFIG"] = _tf_config(spec, r.role, i, tf_port)
            cmd = [sys.executable if c in ("python", "python3") else c for c in r.command]
            key = f"{r.role.lower()}-{i}"
            suffix = f".restart{attempt}" if attempt else ""
            log = open(os.path.join(log_dir, f"{key}{suffix}.log"), "w")
            procs[key] = (subprocess.Popen(cmd, env=env, cwd=cwd, stdout=log, stderr=subprocess.STDOUT), log)
            roles[key] = r
            if is_rank:
                rank += 1
    codes = {}
    # poll every process: the FIRST non-zero exit takes the set down at once (no rank left blocked in a collective
    # waiting for a dead peer until its own timeout)
    live = dict(procs)
    while live:
        for k in list(live):
            c = live[k][0].poll()
            if c is not None:
                codes[k] = c
                live.pop(k)
        if any(c != 0 for c in codes.values()) or (deadline is not None and time.time() >= deadline):
            for k, (p, _) in live.items():
                p.kill()
                p.wait()
                codes[k] = -9
            live = {}
            break
        time.sleep(0.05)
    for _, log in procs.values():
        log.close()
    return codes, roles


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
