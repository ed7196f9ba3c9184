"""Kubernetes helpers: name sanitisation, k8s-model -> JSON conversion, and a minimal pod runner.

Reference: `sdk/python/kfp/compiler/_k8s_helper.py:25-183`. The pod runner talks to the cluster
through `kubectl` (no python kubernetes client is required): create pod -> poll every 5 s ->
delete, with a timeout."""
from __future__ import annotations

import datetime
import json
import re
import subprocess
import time


def sanitize_k8s_name(name: str) -> str:
    return re.sub("-+", "-", re.sub("[^-0-9a-z]+", "-", name.lower())).lstrip("-").rstrip("-")


def convert_k8s_obj_to_json(k8s_obj):
    from ..dsl._pipeline_param import PipelineParam

    if k8s_obj is None:
        return None
    if isinstance(k8s_obj, (float, bool, bytes, str, int)):
        return k8s_obj
    if isinstance(k8s_obj, list):
        return [convert_k8s_obj_to_json(x) for x in k8s_obj]
    if isinstance(k8s_obj, tuple):
        return tuple(convert_k8s_obj_to_json(x) for x in k8s_obj)
    if isinstance(k8s_obj, (datetime.datetime, datetime.date)):
        return k8s_obj.isoformat()
    if isinstance(k8s_obj, PipelineParam):
        if isinstance(k8s_obj.value, str):
            return k8s_obj.value
        return "{{inputs.parameters.%s}}" % k8s_obj.full_name
    if isinstance(k8s_obj, dict):
        d = k8s_obj
    else:
        types = getattr(k8s_obj, "swagger_types", None) or getattr(k8s_obj, "openapi_types", None) or {}
        d = {k8s_obj.attribute_map[a]: getattr(k8s_obj, a) for a in types if getattr(k8s_obj, a) is not None}
    return {k: convert_k8s_obj_to_json(v) for k, v in d.items()}


class K8sHelper:
    sanitize_k8s_name = staticmethod(sanitize_k8s_name)
    convert_k8s_obj_to_json = staticmethod(convert_k8s_obj_to_json)

    def __init__(self, kubectl: str = "kubectl"):
        self.kubectl = kubectl

    def _run(self, *args, input_text: str | None = None) -> str:
        res = subprocess.run([self.kubectl, *args], input=input_text, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"kubectl {' '.join(args)} failed: {res.stderr.strip()}")
        return res.stdout

    def _create_k8s_job(self, pod_spec: dict) -> str:
        out = self._run("create", "-o", "json", "-f", "-", input_text=json.dumps(pod_spec))
        return json.loads(out)["metadata"]["name"]

    def _wait_for_k8s_job(self, pod_name: str, namespace: str, timeout: int) -> str:
        start = time.time()
        while True:
            st = json.loads(self._run("get", "pod", pod_name, "-n", namespace, "-o", "json"))
            phase = st.get("status", {}).get("phase", "Unknown")
            if phase in ("Succeeded", "Failed"):
                return phase
            if time.time() - start > timeout:
                raise TimeoutError(f"pod {pod_name} did not finish in {timeout}s")
            time.sleep(5)

    def _delete_k8s_job(self, pod_name: str, namespace: str) -> None:
        self._run("delete", "pod", pod_name, "-n", namespace)

    def _read_pod_log(self, pod_name: str, namespace: str) -> str:
        return self._run("logs", pod_name, "-n", namespace)

    def run_job(self, yaml_spec: dict, timeout: int = 600) -> bool:
        ns = yaml_spec.get("metadata", {}).get("namespace", "default")
        name = self._create_k8s_job(yaml_spec)
        try:
            phase = self._wait_for_k8s_job(name, ns, timeout)
        finally:
            try:
                self._delete_k8s_job(name, ns)
            except RuntimeError:
                pass
        return phase == "Succeeded"
