"""Cluster execution of compiled pipelines: the Argo workflow-controller's job on Kubernetes, one Pod per step.

The reference deploys Argo (`install-kubeflow/ks_app/vendor/kubeflow/argo/argo.libsonnet:40-91`): its controller turns
every container template of a compiled Workflow into a Pod -- the step's image, command, env, volume mounts (PVCs
from `VolumeOp`, `onprem.mount_pvc`'s `users-pvc`, `sdk/python/kfp/onprem.py:2-22`), resource limits including the
vendor GPU limit `set_gpu_limit` writes (`sdk/python/kfp/dsl/_container_op.py:286-301`; `amd.com/gpu` here), sidecars
-- and applies resource templates (`_volume_op.py:35-142`) with their success / failure conditions. `KubeStepRunner`
is that controller's per-step half for `mifx.kfp.local.LocalWorkflowExecutor`, which keeps the DAG / `when` /
retry / deadline / exit-handler / recursion semantics: `LocalWorkflowExecutor(wf, run_dir, steps=KubeStepRunner(api))`.

Container steps: a Pod named after the workflow and the node, `restartPolicy: Never`, the template's container as
`main` (its resources, volumeMounts, env, securityContext unchanged), the workflow-level volumes its mounts name
(substituted in the step's scope, e.g. `claimName: {{inputs.parameters.create-pvc-name}}`), sidecars, init
containers, nodeSelector / tolerations / affinity, `activeDeadlineSeconds` and the workflow's service account and
image pull secrets. Output parameters leave the pod the way Argo's executor used to hand them over without a
sidecar: `main` runs under a small `sh` wrapper that, after the step exits, writes `name<TAB>base64(file)` lines into
the container's termination message (kubelet: at most 4 KB, so output parameters must stay small; larger outputs
belong on a PVC). The runner polls the pod until `main` has terminated, reads the exit code and the outputs, keeps its
log, and deletes the pod when the step used sidecars (a plain Pod would otherwise never finish) or `pod_gc` asks.
A retry (`retryStrategy.limit`) is a fresh pod, as in Argo.

Resource steps: `create` / `apply` / `patch` / `replace` / `delete` / `get` of the manifest through the REST API,
then `successCondition` / `failureCondition` (Argo's comma-separated `path op value` requirements, ops `==`, `=`,
`!=`, `>`, `<`, `>=`, `<=`, `in (a, b)`, `notin (a, b)`) polled on the live object; output parameters are JSONPath
reads of that object -- so a `VolumeOp` creates its PVC and later steps mount it.

`api` is anything with `get(path)` -> dict | None, `post(path, body)`, `patch(path, body, content_type)`,
`delete(path)` and optionally `get_text(path)` (pod logs): `mifx.launch.operator.KubeApi` in a cluster, an in-memory
fake in tests (tests/test_kfp_kube.py)."""
from __future__ import annotations

import base64
import hashlib
import json
import re
import time

from .executor import NodeStatus, WorkflowError, _substitute

# the step's argv runs as "$@"; afterwards each output parameter file becomes one `name<TAB>base64` line of the
# termination message (MIFX_OUTPUTS: space-separated name=path pairs); the step's exit code is kept
_WRAP = ('"$@"; rc=$?; t="${MIFX_TERMINATION_LOG:-/dev/termination-log}"; : > "$t"; '
         'for kv in $MIFX_OUTPUTS; do n="${kv%%=*}"; p="${kv#*=}"; '
         'if [ -f "$p" ]; then printf "%s\\t%s\\n" "$n" "$(base64 < "$p" | tr -d "\\n")" >> "$t"; fi; done; '
         'exit $rc')
TERMINATION_LIMIT = 4096

_CORE_V1 = {"Pod", "Service", "PersistentVolumeClaim", "Secret", "ConfigMap", "ServiceAccount", "Endpoints", "Event",
            "PersistentVolume", "Namespace", "Node", "ReplicationController", "LimitRange", "ResourceQuota"}
_CLUSTER_SCOPED = {"PersistentVolume", "Namespace", "Node", "ClusterRole", "ClusterRoleBinding", "StorageClass",
                   "CustomResourceDefinition", "VolumeSnapshotClass"}


def plural(kind: str) -> str:
    k = kind.lower()
    if k.endswith("s") and kind != "Endpoints":
        return k + "es"
    if k.endswith("y") and k[-2:-1] not in "aeiou":
        return k[:-1] + "ies"
    return k if kind == "Endpoints" else k + "s"


def resource_path(manifest: dict, namespace: str, name: str | None = None) -> str:
    """REST collection (or object) path of a manifest's kind in `namespace`."""
    api_version, kind = manifest.get("apiVersion", "v1"), manifest.get("kind", "")
    if not kind:
        raise WorkflowError("resource manifest without a kind")
    ns = manifest.get("metadata", {}).get("namespace") or namespace
    base = "/api/v1" if (api_version == "v1" and kind in _CORE_V1) else f"/apis/{api_version}"
    p = f"{base}/{plural(kind)}" if kind in _CLUSTER_SCOPED else f"{base}/namespaces/{ns}/{plural(kind)}"
    return p + (f"/{name}" if name else "")


def json_path(obj, expr: str):
    """The `{.a.b[0].c}` JSONPath subset Argo output parameters use; `{}` is the whole object (as JSON)."""
    e = expr.strip()
    if e.startswith("{") and e.endswith("}"):
        e = e[1:-1]
    e = e.strip().lstrip(".")
    if not e:
        return json.dumps(obj)
    cur = obj
    for part in re.findall(r"[^.\[\]]+|\[\d+\]", e):
        if part.startswith("["):
            i = int(part[1:-1])
            cur = cur[i] if isinstance(cur, list) and i < len(cur) else None
        else:
            cur = cur.get(part) if isinstance(cur, dict) else None
        if cur is None:
            return ""
    return cur if isinstance(cur, str) else json.dumps(cur)


def _field(obj, path: str):
    cur = obj
    for part in path.split("."):
        if not isinstance(cur, dict) or part not in cur:
            return None
        cur = cur[part]
    return cur


def _scalar(v) -> str:
    if isinstance(v, bool):
        return "true" if v else "false"
    return "" if v is None else str(v)


_REQ = re.compile(r"^\s*([\w.\-]+)\s+(notin|in)\s+\((.*)\)\s*$|^\s*([\w.\-]+)\s*(==|!=|>=|<=|=|>|<)\s*(.+?)\s*$")


def condition_holds(obj: dict, cond: str) -> bool:
    """Argo resource success/failure condition: every comma-separated requirement holds on `obj`."""
    reqs = [r for r in re.split(r",(?![^(]*\))", cond or "") if r.strip()]
    if not reqs:
        return False
    for r in reqs:
        m = _REQ.match(r)
        if not m:
            raise WorkflowError(f"cannot parse resource condition {r!r}")
        if m.group(1):  # set membership
            have = _scalar(_field(obj, m.group(1)))
            vals = [x.strip().strip("'\"") for x in m.group(3).split(",")]
            if (have in vals) != (m.group(2) == "in"):
                return False
            continue
        have, op, want = _scalar(_field(obj, m.group(4))), m.group(5), m.group(6).strip("'\"")
        try:
            a, b = float(have), float(want)
        except ValueError:
            if op in (">", "<", ">=", "<="):
                return False
            a, b = have, want
        if not {"==": a == b, "=": a == b, "!=": a != b, ">": a > b, "<": a < b, ">=": a >= b, "<=": a <= b}[op]:
            return False
    return True


def _k8s_name(s: str, limit: int = 63) -> str:
    s = re.sub(r"[^a-z0-9-]+", "-", s.lower()).strip("-")
    return s[:limit].rstrip("-") or "x"


class KubeStepRunner:
    """Runs a workflow executor's container and resource steps on a Kubernetes cluster (see the module doc)."""

    def __init__(self, api, namespace: str = "kubeflow", poll_s: float = 1.0, pod_gc: bool = False,
                 default_image: str | None = None):
        self.api, self.ns, self.poll_s, self.pod_gc = api, namespace, float(poll_s), bool(pod_gc)
        self.default_image = default_image
        self.created: list[str] = []  # object paths, in creation order (the DAG order a test can check)

    # ---- container steps ---------------------------------------------------------------------
    def pod_manifest(self, ex, tmpl: dict, scope: dict, display: str, node: NodeStatus) -> tuple[dict, dict]:
        """(Pod manifest, {output name: path}) of one attempt of a container step."""
        digest = hashlib.sha1(f"{ex.uid}/{display}/{node.attempts}".encode()).hexdigest()[:10]
        name = _k8s_name(f"{ex.name[:40]}-{digest}")
        scope = dict(scope, **{"pod.name": name})
        c = _substitute(tmpl["container"], scope)
        argv = [str(x) for x in (c.get("command") or []) + (c.get("args") or [])]
        if not argv:
            raise WorkflowError(f"{display}: container has no command")
        outs = {}
        for p in (tmpl.get("outputs") or {}).get("parameters", []) or []:
            path = (p.get("valueFrom") or {}).get("path")
            if path is None:
                continue
            if re.search(r"[\s=]", path) or re.search(r"[\s=]", p["name"]):
                raise WorkflowError(f"{display}: output parameter {p['name']} path {path!r} (no spaces or '=')")
            outs[p["name"]] = path
        main = {k: v for k, v in c.items() if k not in ("command", "args")}
        main["name"] = "main"
        main.setdefault("image", self.default_image or "mifx:latest")
        env = [e for e in (c.get("env") or []) if e.get("name") != "MIFX_OUTPUTS"]
        env.append({"name": "MIFX_OUTPUTS", "value": " ".join(f"{k}={v}" for k, v in outs.items())})
        main["env"] = env
        main["command"] = ["sh", "-c", _WRAP, "mifx-step"] + argv
        main.setdefault("terminationMessagePolicy", "File")
        mounts = {m["name"] for m in (c.get("volumeMounts") or [])}
        sidecars = []
        for sc in _substitute(tmpl.get("sidecars") or [], scope):
            sc = dict(sc)
            sc.pop("mirrorVolumeMounts", None)
            mounts |= {m["name"] for m in (sc.get("volumeMounts") or [])}
            sidecars.append(sc)
        inits = _substitute(tmpl.get("initContainers") or [], scope)
        for ic in inits:
            mounts |= {m["name"] for m in (ic.get("volumeMounts") or [])}
        spec_vols = {v["name"]: v for v in (ex.spec.get("volumes") or [])}
        vols = [_substitute(spec_vols[n], scope) for n in sorted(mounts) if n in spec_vols]
        vols += [v for v in _substitute(tmpl.get("volumes") or [], scope) if v["name"] not in spec_vols]
        meta = _substitute(tmpl.get("metadata") or {}, scope)
        labels = {"workflows.argoproj.io/workflow": _k8s_name(ex.name), "mifx.amd.com/step": _k8s_name(tmpl["name"])}
        labels.update(meta.get("labels") or {})
        annotations = {"workflows.argoproj.io/node-name": display}
        annotations.update(meta.get("annotations") or {})
        spec = {"restartPolicy": "Never", "containers": [main] + sidecars}
        if inits:
            spec["initContainers"] = inits
        if vols:
            spec["volumes"] = vols
        for k in ("nodeSelector", "tolerations", "affinity", "schedulerName", "priorityClassName"):
            if tmpl.get(k):
                spec[k] = _substitute(tmpl[k], scope)
        if tmpl.get("activeDeadlineSeconds"):
            spec["activeDeadlineSeconds"] = int(float(tmpl["activeDeadlineSeconds"]))
        if ex.spec.get("serviceAccountName"):
            spec["serviceAccountName"] = ex.spec["serviceAccountName"]
        if ex.spec.get("imagePullSecrets"):
            spec["imagePullSecrets"] = ex.spec["imagePullSecrets"]
        pod = {"apiVersion": "v1", "kind": "Pod",
               "metadata": {"name": name, "namespace": self.ns, "labels": labels, "annotations": annotations},
               "spec": spec}
        return pod, outs

    def _main_status(self, pod: dict) -> dict | None:
        for cs in (pod.get("status") or {}).get("containerStatuses") or []:
            if cs.get("name") == "main":
                return cs
        return None

    def run_container(self, ex, tmpl: dict, scope: dict, display: str, node: NodeStatus) -> dict:
        pod, outs = self.pod_manifest(ex, tmpl, scope, display, node)
        coll = resource_path(pod, self.ns)
        path = f"{coll}/{pod['metadata']['name']}"
        try:
            self.api.post(coll, pod)
        except Exception as e:  # noqa: BLE001 -- the API server refused the pod (quota, admission, ...)
            raise WorkflowError(f"{display}: pod creation failed: {e}") from e
        self.created.append(path)
        node.message = f"pod {pod['metadata']['name']}"
        deadline = None
        if tmpl.get("activeDeadlineSeconds"):
            deadline = time.time() + float(tmpl["activeDeadlineSeconds"]) + 30.0  # (the kubelet enforces it first)
        if ex.deadline:
            deadline = min(deadline, ex.deadline) if deadline else ex.deadline
        term = None
        while True:
            cur = self.api.get(path)
            if cur is None:
                raise WorkflowError(f"{display}: pod {pod['metadata']['name']} disappeared")
            cs = self._main_status(cur)
            term = ((cs or {}).get("state") or {}).get("terminated")
            ph = (cur.get("status") or {}).get("phase")
            if term is not None:
                break
            if ph == "Failed":  # evicted / deadline exceeded before main reported
                st = cur.get("status") or {}
                raise WorkflowError(f"{display}: pod failed: {st.get('reason', '')} {st.get('message', '')}".strip())
            if deadline and time.time() > deadline:
                self._delete(path)
                raise WorkflowError(f"{display}: step exceeded its deadline")
            time.sleep(self.poll_s)
        if hasattr(self.api, "get_text"):
            try:
                node.log = self.api.get_text(f"{path}/log?container=main") or ""
            except Exception:  # noqa: BLE001 -- logs are best effort
                node.log = ""
        if tmpl.get("sidecars") or self.pod_gc:
            self._delete(path)  # sidecars would keep a plain Pod running forever
        code = int(term.get("exitCode", 1))
        if code != 0:
            raise WorkflowError(f"{display}: exit code {code}: {term.get('reason', '')} {node.log[-2000:]}".strip())
        return self._outputs(display, term.get("message") or "", outs)

    @staticmethod
    def _outputs(display: str, message: str, outs: dict) -> dict:
        got = {}
        for line in message.splitlines():
            if "\t" not in line:
                continue
            k, v = line.split("\t", 1)
            try:
                got[k] = base64.b64decode(v.strip(), validate=True).decode().strip()
            except Exception as e:  # noqa: BLE001
                raise WorkflowError(f"{display}: output parameter {k} did not fit the {TERMINATION_LIMIT}-byte "
                                    "termination message (write large outputs to a volume)") from e
        missing = [k for k in outs if k not in got]
        if missing:
            raise WorkflowError(f"{display}: output parameter file(s) not written: "
                                + ", ".join(f"{k} ({outs[k]})" for k in missing))
        return got

    def _delete(self, path: str) -> None:
        try:
            self.api.delete(path)
        except Exception:  # noqa: BLE001 -- already gone
            pass

    # ---- resource steps ----------------------------------------------------------------------
    def run_resource(self, ex, tmpl: dict, scope: dict, display: str) -> dict:
        import yaml

        r = _substitute(tmpl["resource"], scope)
        manifest = yaml.safe_load(r.get("manifest", "")) or {}
        action = r.get("action", "create")
        meta = manifest.setdefault("metadata", {})
        name = meta.get("name")
        coll = resource_path(manifest, self.ns)
        try:
            if action == "create":
                obj = self.api.post(coll, manifest)
                name = (obj or {}).get("metadata", {}).get("name") or name
            elif action in ("apply", "replace"):
                if name is None:
                    raise WorkflowError(f"{display}: {action} needs metadata.name")
                cur = self.api.get(f"{coll}/{name}")
                obj = self.api.post(coll, manifest) if cur is None else \
                    self.api.patch(f"{coll}/{name}", manifest, "application/merge-patch+json")
            elif action == "patch":
                ctype = {"json": "application/json-patch+json", "merge": "application/merge-patch+json",
                         "strategic": "application/strategic-merge-patch+json"}[r.get("mergeStrategy") or "strategic"]
                obj = self.api.patch(f"{coll}/{name}", manifest, ctype)
            elif action == "delete":
                self.api.delete(f"{coll}/{name}")
                obj = manifest
            elif action == "get":
                obj = self.api.get(f"{coll}/{name}")
                if obj is None:
                    raise WorkflowError(f"{display}: {coll}/{name} not found")
            else:
                raise WorkflowError(f"{display}: unsupported resource action {action!r}")
        except WorkflowError:
            raise
        except Exception as e:  # noqa: BLE001 -- refused by the API server
            raise WorkflowError(f"{display}: {action} {manifest.get('kind')}: {e}") from e
        path = f"{coll}/{name}"
        if action != "delete":
            self.created.append(path)
        succ, fail = r.get("successCondition"), r.get("failureCondition")
        if action != "delete" and (succ or fail):
            deadline = ex.deadline
            if tmpl.get("activeDeadlineSeconds"):
                d2 = time.time() + float(tmpl["activeDeadlineSeconds"])
                deadline = min(deadline, d2) if deadline else d2
            while True:
                obj = self.api.get(path) or {}
                if fail and condition_holds(obj, fail):
                    raise WorkflowError(f"{display}: failure condition {fail!r} holds on {path}")
                if not succ or condition_holds(obj, succ):
                    break
                if deadline and time.time() > deadline:
                    raise WorkflowError(f"{display}: success condition {succ!r} not reached before the deadline")
                time.sleep(self.poll_s)
        elif action != "delete":
            obj = self.api.get(path) or obj
        outs = {}
        for p in (tmpl.get("outputs") or {}).get("parameters", []) or []:
            jp = (p.get("valueFrom") or {}).get("jsonPath")
            if jp is not None:
                outs[p["name"]] = json_path(obj, jp)
        return outs


def wrapper_command(argv: list[str]) -> list[str]:
    """The argv a step's main container runs (for inspection / local checks of the output hand-over)."""
    return ["sh", "-c", _WRAP, "mifx-step"] + list(argv)


__all__ = ["KubeStepRunner", "condition_holds", "json_path", "plural", "resource_path", "wrapper_command"]
