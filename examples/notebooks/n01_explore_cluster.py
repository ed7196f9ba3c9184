"""Notebook 01_Explore_Kubernetes_Cluster (reference `notebooks/01_Explore_Kubernetes_Cluster.ipynb`
L11-29: `kubectl get nodes/pods`, `kubectl describe`, `kubectl logs`) for the mifx stack. The cluster view is
the pipelines backend (`local://<dir>` or a `mifx-pipelines-api` URL) plus this host's accelerators:

* get nodes    -> the visible MI355X GPUs (arch, CUs, HBM) from `mifx.utils.env.report`
* get pods     -> pipeline runs and their status (`Client.list_runs`)
* describe     -> the newest run's workflow: one line per step with its phase
* logs         -> each step's captured stdout/stderr (`<run_data>/<run id>/.../log.txt` for the local backend)
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import mifx.kfp as kfp  # noqa: E402
from mifx.utils import env  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=None, help="local://<dir> or pipelines API URL (default: local://<tmp>/kfp)")
    ap.add_argument("--tail", type=int, default=20, help="log lines shown per step")
    a = ap.parse_args(argv)
    host = a.host or f"local://{os.path.join(tempfile.gettempdir(), 'mifx_n08', 'kfp')}"
    rep = env.report()
    print("NODES (accelerators)")
    for g in rep["gpus"] or [{"name": "cpu-only host"}]:
        print("  ", json.dumps(g))
    client = kfp.Client(host=host)
    runs = client.list_runs(page_size=100, sort_by="created_at des").runs or []
    print(f"RUNS ({len(runs)})")
    for r in runs:
        print(f"   {r['id']}  {r['status']:<10} {r['name']}")
    out = {"gpus": rep["gpus"], "runs": runs, "steps": {}, "logs": {}}
    if not runs:
        return out
    latest = runs[0]["id"]
    wf = json.loads(client.get_run(latest).pipeline_runtime.workflow_manifest)
    print(f"DESCRIBE run {latest}")
    for name, node in ((wf.get("status") or {}).get("nodes") or {}).items():
        phase = node.get("phase") if isinstance(node, dict) else node
        out["steps"][name] = phase
        print(f"   {name:<40} {phase}")
    if host.startswith("local://"):
        root = os.path.join(host[len("local://"):], "run_data", latest)
        for path in sorted(glob.glob(os.path.join(root, "**", "log.txt"), recursive=True)):
            with open(path) as f:
                lines = f.read().splitlines()
            step = os.path.relpath(os.path.dirname(path), root)
            out["logs"][step] = lines
            print(f"LOGS {step}")
            for ln in lines[-a.tail:]:
                print("   ", ln)
    return out


if __name__ == "__main__":
    main()
