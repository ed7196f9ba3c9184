"""Data-parallel Trainer runs: one process per GPU, launched by the Trainer component itself.

The reference's distributed training is a Kubernetes job the user writes by hand (TFJob with 3 workers,
`notebooks/training-jobs/distributed-tensorflow-training-job.yaml:1-18`; the parameter-server prototype
`install-kubeflow/ks_app/vendor/kubeflow/examples/prototypes/tf-job-simple-v1beta2.jsonnet:22-74`) around the
same `trainer_fn(hparams, schema)` contract the TFX Trainer calls (`airflow-dags/taxi_utils.py:285-356`). Here
`Trainer(custom_config={"num_gpus": N})` does it: the executor writes a run spec, starts N ranks of

    python -m mifx.trainer.distributed <spec.json>

with torchrun-style env (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) BEFORE anything
in the parent touches the GPU on their behalf, and waits. Every rank initialises torch.distributed (RCCL over
xGMI on GPUs, gloo on CPU), calls the user's `trainer_fn` and `train_and_evaluate`; the estimator sees the
process group and trains its shard of every global batch (`estimator.shard_records`) with the gradient
exchanged every step (W&D: the one-shot xGMI exchange inside the step's hipGraph, else direct RCCL; CPU: the
bucketed all-reduce). Rank 0 checkpoints, evaluates, exports and writes `result.json`; a failing rank takes
the job down (restartPolicy Never semantics, as the reference's TFJob).

`MIFX_SHARED_GPU=1` (with `MIFX_DIST_BACKEND=gloo`) rehearses the multi-rank flow with every rank on cuda:0."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

RESULT = "result.json"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(spec: dict, num_procs: int, work_dir: str, timeout: float | None = None) -> dict:
    """Run `num_procs` ranks of the spec and return rank 0's result dict. Raises if any rank fails."""
    os.makedirs(work_dir, exist_ok=True)
    path = os.path.join(work_dir, "dp_spec.json")
    with open(path, "w") as f:
        json.dump(spec, f, default=str)
    run_ranks(["-m", "mifx.trainer.distributed", path], num_procs, work_dir, timeout)
    with open(os.path.join(work_dir, RESULT)) as f:
        return json.load(f)


def run_ranks(args: list, num_procs: int, work_dir: str, timeout: float | None = None) -> None:
    """Start `python <args>` once per rank (torchrun-style env, logs in work_dir/rank<r>.log) and wait; a failing
    rank kills the others and raises with every rank's log tail."""
    os.makedirs(work_dir, exist_ok=True)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    port = _free_port()
    procs = []
    for r in range(num_procs):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(num_procs),
                    "LOCAL_WORLD_SIZE": str(num_procs), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
                    "PYTHONPATH": os.pathsep.join([root, env.get("PYTHONPATH", "")]).rstrip(os.pathsep)})
        log = open(os.path.join(work_dir, f"rank{r}.log"), "w")
        procs.append((subprocess.Popen([sys.executable] + list(args), env=env, stdout=log,
                                       stderr=subprocess.STDOUT), log))
    deadline = time.time() + timeout if timeout else None
    codes = [None] * num_procs
    try:
        while any(c is None for c in codes):
            for i, (p, _) in enumerate(procs):
                if codes[i] is None:
                    codes[i] = p.poll()
            if any(c not in (None, 0) for c in codes):
                break  # a failed rank takes the job down
            if deadline and time.time() > deadline:
                break
            time.sleep(0.05)
    finally:
        for i, (p, log) in enumerate(procs):
            if p.poll() is None:
                p.kill()
                p.wait()
            codes[i] = p.returncode
            log.close()
    if any(c != 0 for c in codes):
        tails = []
        for r in range(num_procs):
            with open(os.path.join(work_dir, f"rank{r}.log")) as f:
                tails.append(f"--- rank {r} (exit {codes[r]}) ---\n" + "".join(f.readlines()[-25:]))
        raise RuntimeError("data-parallel Trainer failed:\n" + "\n".join(tails))


def run_trainer_fn(module_file: str, hp_values: dict, schema_uri: str, out_dir: str) -> dict:
    """What one Trainer run does in a process (rank or single): trainer_fn -> train_and_evaluate -> exports.
    Returns {"eval": metrics, "exports": [...], "train_examples_per_sec": ...} (empty metrics off rank 0)."""
    from ..components.statistics import load_schema_from_artifact
    from ..transform import import_module_file
    from .estimator import HParams, train_and_evaluate

    trainer_fn = import_module_file(module_file, "trainer_fn")
    hp = HParams(**hp_values)
    spec = trainer_fn(hp, load_schema_from_artifact(schema_uri))
    est = spec["estimator"]
    try:
        metrics, exports = train_and_evaluate(est, spec["train_spec"], spec["eval_spec"])
        if getattr(est, "rank", 0) == 0 and spec.get("eval_input_receiver_fn") is not None:
            est.export_saved_model(hp.eval_model_dir, spec["eval_input_receiver_fn"])
        dump = (hp_values.get("custom_config") or {}).get("dump_replicas_dir")
        if dump:  # every rank's final weights (replica-agreement checks)
            import torch

            os.makedirs(dump, exist_ok=True)
            torch.save({k: v.detach().cpu() for k, v in est.model.state_dict().items()},
                       os.path.join(dump, f"replica{getattr(est, 'rank', 0)}.pt"))
    finally:
        if hasattr(est, "close"):
            est.close()
    return {"eval": metrics, "exports": exports, "train_examples_per_sec": getattr(est, "examples_per_sec", None),
            "world_size": getattr(est, "world", 1), "global_step": getattr(est, "global_step", None)}


def worker_main(spec_path: str) -> int:
    with open(spec_path) as f:
        spec = json.load(f)
    import torch

    from ..parallel import dist as mdist

    spec.setdefault("hparams", {})
    cpu = spec["hparams"].get("device") == "cpu" or not torch.cuda.is_available()
    env = mdist.init("gloo" if cpu else None)
    try:
        hp = dict(spec["hparams"])
        if hp.get("device") in (None, "cuda") and torch.cuda.is_available():
            hp["device"] = "cuda"  # the estimator picks cuda:LOCAL_RANK (cuda:0 under MIFX_SHARED_GPU)
        target = spec.get("target")
        if target:  # another per-rank entry point (e.g. the BERT tensor-parallel Trainer): module:function(spec)
            import importlib

            mod, _, fn = target.partition(":")
            res = getattr(importlib.import_module(mod), fn)(spec)
        else:
            res = run_trainer_fn(spec["module_file"], hp, spec["schema_uri"], spec["out_dir"])
        if env.rank == 0:
            with open(os.path.join(spec["work_dir"], RESULT), "w") as f:
                json.dump(res, f, default=float)
    finally:
        mdist.shutdown()
    return 0


if __name__ == "__main__":
    raise SystemExit(worker_main(sys.argv[1]))
