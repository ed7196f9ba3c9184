from __future__ import annotations

import base64
import multiprocessing as mp
import os
import tempfile

import cloudpickle

_ENTRY = """import base64, pickle, sys
fn = pickle.loads(base64.b64decode(open(sys.argv[1]).read()))
res = fn()
print("fairing result:", res)
"""


def _child(payload: bytes, q):
    try:
        fn = cloudpickle.loads(payload)
        q.put(("ok", fn()))
    except BaseException as e:  # noqa: BLE001 - reported to the parent
        q.put(("err", repr(e)))


class Config:
    def __init__(self):
        self.builder = {"name": "append", "base_image": "rocm/pytorch:latest", "registry": None, "push": False}
        self.deployer = {"name": "local", "namespace": "kubeflow", "gpus": 0, "pod_spec_mutators": []}
        self.model = None

    def set_builder(self, name: str = "append", base_image: str | None = None, registry: str | None = None,
                    push: bool = True, **kw) -> None:
        self.builder = {"name": name, "base_image": base_image or self.builder["base_image"], "registry": registry,
                        "push": push, **kw}
        if name == "cluster" and self.deployer["name"] == "local":
            self.deployer["name"] = "job"

    def set_deployer(self, name: str = "job", namespace: str = "kubeflow", gpus: int = 0, **kw) -> None:
        self.deployer = {"name": name, "namespace": namespace, "gpus": gpus, "pod_spec_mutators": [], **kw}

    def set_model(self, model) -> None:
        self.model = model

    # ---- execution ------------------------------------------------------------------------
    def _run_callable(self, fn):
        if self.deployer["name"] == "local":
            ctx = mp.get_context("spawn")
            q = ctx.Queue()
            p = ctx.Process(target=_child, args=(cloudpickle.dumps(fn), q))
            p.start()
            status, val = q.get()
            p.join()
            if status != "ok":
                raise RuntimeError(f"remote function failed: {val}")
            return val
        return self.submit_job(fn)

    def fn(self, func):
        def wrapped(*args, **kwargs):
            return self._run_callable(lambda: func(*args, **kwargs))

        wrapped.__name__ = getattr(func, "__name__", "fairing_fn")
        return wrapped

    def run(self):
        if self.model is None:
            raise ValueError("set_model() first")
        m = self.model
        return self._run_callable(lambda: m.train())

    # ---- cluster path -----------------------------------------------------------------------
    def image_name(self) -> str:
        reg = self.builder.get("registry") or "local"
        return f"{reg}/fairing-job:latest"

    def build_context(self, fn, out_dir: str) -> str:
        os.makedirs(out_dir, exist_ok=True)
        with open(os.path.join(out_dir, "fn.pkl.b64"), "w") as f:
            f.write(base64.b64encode(cloudpickle.dumps(fn)).decode())
        with open(os.path.join(out_dir, "entry.py"), "w") as f:
            f.write(_ENTRY)
        with open(os.path.join(out_dir, "Dockerfile"), "w") as f:
            f.write(f"FROM {self.builder['base_image']}\nRUN pip3 install cloudpickle\nCOPY . /app/\n"
                    "WORKDIR /app\nENTRYPOINT [\"python3\", \"/app/entry.py\", \"/app/fn.pkl.b64\"]\n")
        return out_dir

    def job_manifest(self, name: str = "fairing-job") -> dict:
        c = {"name": name, "image": self.image_name(), "env": [{"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"}]}
        if self.deployer.get("gpus"):
            c["resources"] = {"limits": {"amd.com/gpu": str(self.deployer["gpus"])}}
        return {"apiVersion": "batch/v1", "kind": "Job",
                "metadata": {"generateName": name + "-", "namespace": self.deployer["namespace"]},
                "spec": {"backoffLimit": 0, "template": {"spec": {"restartPolicy": "Never", "containers": [c]}}}}

    def submit_job(self, fn):
        from ..kfp.compiler._component_builder import ImageBuilder
        from ..kfp.compiler._k8s_helper import K8sHelper

        with tempfile.TemporaryDirectory() as d:
            self.build_context(fn, d)
            if self.builder.get("push", True) and self.builder.get("staging"):
                ImageBuilder(self.builder["staging"], self.image_name()).build_image_from_dockerfile(
                    os.path.join(d, "Dockerfile"), 600, self.deployer["namespace"])
        return K8sHelper().run_job(self.job_manifest(), timeout=self.deployer.get("timeout", 3600))


config = Config()
