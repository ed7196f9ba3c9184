"""Local Argo-workflow executor: runs a compiled pipeline (the compiler's Workflow dict) on this host.

This is the Argo controller's role for the pipelines the compiler emits (`sdk/python/kfp/compiler/compiler.py`
emits the Workflow; the reference's Argo executes it in-cluster). Semantics implemented: `dag` templates
(dependencies, `when` conditions, DAG output parameters), `container` and `resource` templates through a step runner
-- by default on this host (containers as host subprocesses: the image is recorded, not pulled; resource manifests
recorded), with `steps=mifx.kfp.local.kube.KubeStepRunner(api)` on a Kubernetes cluster (one Pod per step with its
image, volumes / PVCs, `amd.com/gpu` limits and sidecars; resource templates applied with their success / failure
conditions) -- `{{inputs.parameters.*}}`,
`{{tasks.*.outputs.parameters.*}}`, `{{workflow.parameters.*}}` / name / uid substitution,
`retryStrategy.limit`, `activeDeadlineSeconds`, `onExit`, recursion (graph components), and
parallel execution of independent tasks.

Every absolute path a container template names as an output (`valueFrom.path`, artifact paths) is
remapped into a private sandbox per step by rewriting the command line, so steps that all write
`/tmp/output` or `/outputs/<name>/data` don't collide and nothing outside the run directory is
touched."""
from __future__ import annotations

import concurrent.futures as cf
import json
import os
import re
import subprocess
import threading
import time
import hashlib
import uuid
from dataclasses import dataclass, field

_REF = re.compile(r"\{\{([^{}]+)\}\}")


class WorkflowError(RuntimeError):
    pass


@dataclass
class NodeStatus:
    name: str
    template: str
    phase: str = "Pending"  # Pending | Running | Succeeded | Failed | Skipped | Error
    started: float = 0.0
    finished: float = 0.0
    outputs: dict = field(default_factory=dict)
    message: str = ""
    log: str = ""
    attempts: int = 0
    children: list = field(default_factory=list)

    def to_dict(self):
        return {"name": self.name, "templateName": self.template, "phase": self.phase, "startedAt": self.started,
                "finishedAt": self.finished, "outputs": {"parameters": [{"name": k, "value": v}
                                                                        for k, v in self.outputs.items()]},
                "message": self.message, "attempts": self.attempts, "children": list(self.children)}


def _substitute(obj, scope: dict):
    if isinstance(obj, str):
        return _REF.sub(lambda m: str(scope[m.group(1).strip()]) if m.group(1).strip() in scope else m.group(0), obj)
    if isinstance(obj, list):
        return [_substitute(x, scope) for x in obj]
    if isinstance(obj, dict):
        return {k: _substitute(v, scope) for k, v in obj.items()}
    return obj


def _num(x: str):
    try:
        return float(x)
    except (TypeError, ValueError):
        return None


def evaluate_when(expr: str) -> bool:
    """Argo `when`: `<lhs> <op> <rhs>` (numeric compare when both sides are numbers), `&&`, `||`."""
    expr = expr.strip()
    for joiner, fn in (("||", any), ("&&", all)):
        if joiner in expr:
            return fn(evaluate_when(p) for p in expr.split(joiner))
    m = re.match(r"^(.*?)\s*(==|!=|>=|<=|>|<)\s*(.*)$", expr)
    if not m:
        return expr.lower() in ("true", "1")
    lhs, op, rhs = (s.strip().strip("'\"") for s in m.groups())
    ln, rn = _num(lhs), _num(rhs)
    a, b = (ln, rn) if ln is not None and rn is not None else (lhs, rhs)
    return {"==": a == b, "!=": a != b, ">": a > b, "<": a < b, ">=": a >= b, "<=": a <= b}[op]


class LocalWorkflowExecutor:
    """Execute one Workflow dict. `run()` returns the final workflow status dict."""

    def __init__(self, workflow: dict, run_dir: str, arguments: dict | None = None, max_parallel: int = 4,
                 env: dict | None = None, timeout: float | None = None, max_depth: int = 64, steps=None):
        """steps: runner of the container / resource steps (`run_container(ex, tmpl, scope, display, node)`,
        `run_resource(ex, tmpl, scope, display)`, e.g. kube.KubeStepRunner); None runs them on this host."""
        self.steps = steps
        self.wf = workflow
        self.spec = workflow["spec"]
        self.templates = {t["name"]: t for t in self.spec["templates"]}
        self.run_dir = os.path.abspath(run_dir)
        os.makedirs(self.run_dir, exist_ok=True)
        self.params = {p["name"]: p.get("value") for p in self.spec.get("arguments", {}).get("parameters", [])}
        for k, v in (arguments or {}).items():  # names as in the compiled spec (k8s-sanitised)
            key = k if k in self.params else re.sub("-+", "-", re.sub("[^-0-9a-z]+", "-", k.lower())).strip("-")
            self.params[key] = str(v)
        missing = [k for k, v in self.params.items() if v is None]
        if missing:
            raise WorkflowError(f"missing values for workflow parameters: {missing}")
        self.name = workflow.get("metadata", {}).get("name") or \
            workflow.get("metadata", {}).get("generateName", "workflow-") + uuid.uuid4().hex[:5]
        self.uid = str(uuid.uuid4())
        self.max_parallel = max_parallel
        self.env = env
        self.deadline = time.time() + timeout if timeout else None
        self.max_depth = max_depth
        self.nodes: dict[str, NodeStatus] = {}
        self._lock = threading.Lock()
        self._slots = threading.BoundedSemaphore(max(1, max_parallel))  # concurrent container steps
        self._seq = 0
        self._wf_status = None  # set while the exit handler runs

    # ---- helpers -----------------------------------------------------------------------------
    def _global_scope(self) -> dict:
        s = {f"workflow.parameters.{k}": v for k, v in self.params.items()}
        s.update({"workflow.name": self.name, "workflow.uid": self.uid,
                  "workflow.namespace": getattr(self.steps, "ns", "local")})
        if self._wf_status is not None:
            s["workflow.status"] = self._wf_status
        return s

    def _new_node(self, display: str, template: str) -> NodeStatus:
        with self._lock:
            self._seq += 1
            node_id = f"{self.name}-{self._seq}"
            n = NodeStatus(name=display, template=template)
            self.nodes[node_id] = n
        return n

    def _inputs_scope(self, tmpl: dict, args: dict) -> dict:
        scope = self._global_scope()
        for p in tmpl.get("inputs", {}).get("parameters", []) or []:
            if p["name"] in args:
                v = args[p["name"]]
            elif "value" in p:
                v = p["value"]
            elif "default" in p:
                v = p["default"]
            else:
                raise WorkflowError(f"template {tmpl['name']}: no value for input parameter {p['name']}")
            scope[f"inputs.parameters.{p['name']}"] = v
        return scope

    # ---- execution -----------------------------------------------------------------------------
    def run(self) -> dict:
        started = time.time()
        phase, message = "Succeeded", ""
        try:
            # Argo binds workflow arguments to the entrypoint's input parameters by name
            self._exec_template(self.spec["entrypoint"], dict(self.params), self.name, 0)
        except WorkflowError as e:
            phase, message = "Failed", str(e)
        exit_phase = None
        if self.spec.get("onExit"):
            self._wf_status = phase
            try:
                self._exec_template(self.spec["onExit"], {}, self.name + ".onExit", 0)
                exit_phase = "Succeeded"
            except WorkflowError as e:
                exit_phase = "Failed"
                if phase == "Succeeded":
                    phase, message = "Failed", f"exit handler failed: {e}"
        status = {"phase": phase, "message": message, "startedAt": started, "finishedAt": time.time(),
                  "nodes": {k: v.to_dict() for k, v in self.nodes.items()}, "onExitPhase": exit_phase}
        with open(os.path.join(self.run_dir, "status.json"), "w") as f:
            json.dump(status, f, indent=1, default=str)
        return status

    def _check_deadline(self):
        if self.deadline and time.time() > self.deadline:
            raise WorkflowError("workflow deadline exceeded")

    def _exec_template(self, name: str, args: dict, display: str, depth: int, extra_scope: dict | None = None) -> dict:
        if depth > self.max_depth:
            raise WorkflowError(f"maximum recursion depth {self.max_depth} exceeded at {display}")
        self._check_deadline()
        tmpl = self.templates.get(name)
        if tmpl is None:
            raise WorkflowError(f"template {name} not found")
        scope = self._inputs_scope(tmpl, args)
        if extra_scope:
            scope.update(extra_scope)
        node = self._new_node(display, name)
        node.started, node.phase = time.time(), "Running"
        retries = int((tmpl.get("retryStrategy") or {}).get("limit", 0) or 0)
        try:
            for attempt in range(retries + 1):
                node.attempts = attempt + 1
                try:
                    if "dag" in tmpl:
                        outputs = self._exec_dag(tmpl, scope, display, depth, node)
                    elif "container" in tmpl and self.steps is not None:
                        with self._slots:
                            outputs = self.steps.run_container(self, tmpl, scope, display, node)
                    elif "container" in tmpl:
                        outputs = self._exec_container(tmpl, scope, display, node)
                    elif "resource" in tmpl and self.steps is not None:
                        outputs = self.steps.run_resource(self, tmpl, scope, display)
                    elif "resource" in tmpl:
                        outputs = self._exec_resource(tmpl, scope, display)
                    else:
                        raise WorkflowError(f"template {name}: unsupported template kind")
                    break
                except WorkflowError:
                    if attempt == retries:
                        raise
        except WorkflowError as e:
            node.phase, node.message, node.finished = "Failed", str(e), time.time()
            raise
        node.outputs, node.phase, node.finished = outputs, "Succeeded", time.time()
        return outputs

    def _exec_dag(self, tmpl: dict, scope: dict, display: str, depth: int, node: NodeStatus) -> dict:
        tasks = {t["name"]: t for t in tmpl["dag"]["tasks"]}
        state: dict[str, str] = {}
        task_scope = dict(scope)
        futures: dict = {}
        failure = None
        while len(state) < len(tasks):
            progressed = False
            for tname, t in tasks.items():
                if tname in state or tname in futures:
                    continue
                deps = t.get("dependencies") or []
                if any(d not in state for d in deps):
                    continue
                if failure is not None or any(state[d] == "Failed" for d in deps):
                    state[tname] = "Omitted"
                    progressed = True
                    continue
                targs = {p["name"]: p.get("value") for p in (t.get("arguments") or {}).get("parameters", []) or []}
                targs = _substitute(targs, task_scope)
                when = t.get("when")
                if when is not None and not evaluate_when(_substitute(when, task_scope)):
                    state[tname] = "Skipped"
                    sk = self._new_node(f"{display}.{tname}", t["template"])
                    sk.phase = "Skipped"
                    node.children.append(sk.name)
                    progressed = True
                    continue
                node.children.append(f"{display}.{tname}")
                futures[tname] = _spawn(self._exec_template, t["template"], targs, f"{display}.{tname}", depth + 1)
                progressed = True
            if futures:
                done, _ = cf.wait(list(futures.values()), return_when=cf.FIRST_COMPLETED)
                for tname in [k for k, f in futures.items() if f in done]:
                    f = futures.pop(tname)
                    try:
                        outs = f.result()
                        state[tname] = "Succeeded"
                        for k, v in outs.items():
                            task_scope[f"tasks.{tname}.outputs.parameters.{k}"] = v
                    except WorkflowError as e:
                        state[tname] = "Failed"
                        failure = failure or e
                progressed = True
            if not progressed:
                raise WorkflowError(f"dag {tmpl['name']}: dependency cycle or missing task")
        if failure is not None:
            raise WorkflowError(f"dag {tmpl['name']} failed: {failure}")
        outs = {}
        for p in (tmpl.get("outputs") or {}).get("parameters", []) or []:
            expr = (p.get("valueFrom") or {}).get("parameter")
            if expr is not None:
                outs[p["name"]] = _substitute(expr, task_scope)
        return outs

    def _sandbox_paths(self, tmpl: dict, sandbox: str) -> dict:
        paths = []
        outs = tmpl.get("outputs") or {}
        for p in outs.get("parameters", []) or []:
            if (p.get("valueFrom") or {}).get("path"):
                paths.append(p["valueFrom"]["path"])
        for a in outs.get("artifacts", []) or []:
            if a.get("path"):
                paths.append(a["path"])
        return {p: os.path.join(sandbox, p.lstrip("/")) for p in sorted(set(paths), key=len, reverse=True)}

    def _exec_container(self, tmpl: dict, scope: dict, display: str, node: NodeStatus) -> dict:
        pod = re.sub(r"[^A-Za-z0-9_.-]+", "_", display) + f"-{node.attempts}"
        if len(pod) > 120:  # deep recursion grows the display path past the file-name limit: keep it unique
            pod = pod[:48] + "-" + hashlib.sha1(pod.encode()).hexdigest()[:16] + pod[-48:]
        scope = dict(scope, **{"pod.name": pod})
        c = _substitute(tmpl["container"], scope)
        sandbox = os.path.join(self.run_dir, "steps", pod)
        os.makedirs(sandbox, exist_ok=True)
        remap = self._sandbox_paths(tmpl, sandbox)

        def fix(s: str) -> str:
            for src, dst in remap.items():
                s = s.replace(src, dst)
            return s

        argv = [fix(str(x)) for x in (c.get("command") or []) + (c.get("args") or [])]
        if not argv:
            raise WorkflowError(f"{display}: container has no command")
        for dst in remap.values():
            os.makedirs(os.path.dirname(dst), exist_ok=True)
        env = dict(os.environ if self.env is None else self.env)
        for e in c.get("env") or []:
            if "value" in e:
                env[e["name"]] = str(e["value"])
        env["MIFX_KFP_SANDBOX"] = sandbox
        timeout = tmpl.get("activeDeadlineSeconds")
        if self.deadline:
            left = max(1.0, self.deadline - time.time())
            timeout = min(float(timeout), left) if timeout else left
        try:
            with self._slots:
                    res = subprocess.run(argv, cwd=sandbox, env=env, capture_output=True, text=True,
                                     timeout=float(timeout) if timeout else None)
        except subprocess.TimeoutExpired as e:
            raise WorkflowError(f"{display}: step exceeded its deadline") from e
        except FileNotFoundError as e:
            raise WorkflowError(f"{display}: {e}") from e
        node.log = res.stdout + res.stderr
        with open(os.path.join(sandbox, "log.txt"), "w") as f:
            f.write(node.log)
        with open(os.path.join(sandbox, "step.json"), "w") as f:
            json.dump({"image": c.get("image"), "argv": argv, "returncode": res.returncode}, f, indent=1)
        if res.returncode != 0:
            raise WorkflowError(f"{display}: exit code {res.returncode}: {res.stderr.strip()[-2000:]}")
        outs = {}
        for p in (tmpl.get("outputs") or {}).get("parameters", []) or []:
            path = (p.get("valueFrom") or {}).get("path")
            if path is None:
                continue
            try:
                with open(remap[path]) as f:
                    outs[p["name"]] = f.read().strip()
            except FileNotFoundError as e:
                raise WorkflowError(f"{display}: output parameter {p['name']} file {path} was not written") from e
        return outs

    def _exec_resource(self, tmpl: dict, scope: dict, display: str) -> dict:
        r = _substitute(tmpl["resource"], scope)
        import yaml

        manifest = yaml.safe_load(r.get("manifest", "")) or {}
        meta = manifest.get("metadata", {})
        name = meta.get("name") or (meta.get("generateName", "resource-") + uuid.uuid4().hex[:5])
        manifest.setdefault("metadata", {})["name"] = name
        d = os.path.join(self.run_dir, "resources")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, re.sub(r"[^A-Za-z0-9_.-]+", "_", display) + ".json"), "w") as f:
            json.dump({"action": r.get("action"), "manifest": manifest}, f, indent=1)
        outs = {}
        for p in (tmpl.get("outputs") or {}).get("parameters", []) or []:
            jp = (p.get("valueFrom") or {}).get("jsonPath", "")
            cur = manifest
            for part in [x for x in jp.lstrip("{").rstrip("}").lstrip(".").split(".") if x]:
                cur = cur.get(part, "") if isinstance(cur, dict) else ""
            outs[p["name"]] = cur if isinstance(cur, str) else json.dumps(cur)
        return outs


def _spawn(fn, *a) -> cf.Future:
    """Run `fn(*a)` on its own thread. DAG nodes only orchestrate (they block on children), so they
    must not hold slots of a bounded pool; container concurrency is bounded by `_slots` instead."""
    fut: cf.Future = cf.Future()

    def body():
        try:
            fut.set_result(fn(*a))
        except BaseException as e:  # noqa: BLE001 - delivered to the waiting parent
            fut.set_exception(e)

    threading.Thread(target=body, daemon=True).start()
    return fut


def run_workflow(workflow: dict, run_dir: str, arguments: dict | None = None, **kw) -> dict:
    return LocalWorkflowExecutor(workflow, run_dir, arguments, **kw).run()
