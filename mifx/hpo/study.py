"""StudyJob-style hyper-parameter search.

Reference: `notebooks/hyperparameter-tuning/random-search-job.yaml:1-60` (Katib v1alpha1 StudyJob:
maximize `Validation-accuracy` to goal 0.99; `requestcount: 4` rounds of `requestNumber: 3`
random suggestions over --lr [0.01, 0.03] (double), --num-layers [2, 5] (int), --optimizer
{sgd, adam, ftrl} (categorical); each trial is a worker Job running the training command with
`name=value` arguments; the metrics collector parses `name=value` lines from the worker log).

MI355X-first: trials of one request run concurrently, each pinned to its own GPU through
`HIP_VISIBLE_DEVICES` (round-robin over the node's GPUs), so a 3-trial request fills 3 of 8
MI355X instead of queueing on one device. Trials can also be in-process Python callables."""
from __future__ import annotations

import concurrent.futures as cf
import itertools
import json
import math
import os
import random
import re
import subprocess
import time
from dataclasses import dataclass, field

import yaml

_METRIC = re.compile(r"([A-Za-z][\w\-./]*)\s*[=:]\s*([-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?)")


def parse_metrics(text: str, names: list[str]) -> dict:
    """Last value of each `name=value` (or `name: value`) occurrence in a worker log."""
    out = {}
    for m in _METRIC.finditer(text):
        if m.group(1) in names:
            out[m.group(1)] = float(m.group(2))
    return out


@dataclass
class ParameterConfig:
    name: str
    parametertype: str  # double | int | categorical | discrete
    min: float | None = None
    max: float | None = None
    values: list = field(default_factory=list)
    step: float | None = None

    @staticmethod
    def from_dict(d: dict) -> "ParameterConfig":
        f = d.get("feasible", {})
        return ParameterConfig(d["name"], d["parametertype"], float(f["min"]) if "min" in f else None,
                               float(f["max"]) if "max" in f else None, list(f.get("list", [])),
                               float(f["step"]) if "step" in f else None)

    def sample(self, rng: random.Random):
        if self.parametertype == "double":
            return rng.uniform(self.min, self.max)
        if self.parametertype == "int":
            return rng.randint(int(self.min), int(self.max))
        return rng.choice(self.values)

    def grid(self, points: int = 3) -> list:
        if self.parametertype in ("categorical", "discrete"):
            return list(self.values)
        if self.parametertype == "int":
            return list(range(int(self.min), int(self.max) + 1, int(self.step or 1)))
        if self.step:
            n = int(math.floor((self.max - self.min) / self.step + 1e-9)) + 1
            return [self.min + i * self.step for i in range(n)]
        return [self.min + (self.max - self.min) * i / (points - 1) for i in range(points)]


@dataclass
class StudySpec:
    name: str
    optimization: str  # maximize | minimize
    objective: str
    goal: float | None
    request_count: int
    request_number: int
    metrics: list
    parameters: list
    algorithm: str = "random"
    command: list = field(default_factory=list)
    seed: int = 0

    @staticmethod
    def from_dict(d: dict) -> "StudySpec":
        s = d.get("spec", d)
        sug = s.get("suggestionSpec", {})
        cmd = s.get("workerSpec", {}).get("command", [])
        if not cmd and "goTemplate" in s.get("workerSpec", {}):
            cmd = _command_from_go_template(s["workerSpec"]["goTemplate"].get("rawTemplate", ""))
        return StudySpec(name=s.get("studyName", d.get("metadata", {}).get("name", "study")),
                         optimization=s.get("optimizationtype", "maximize"),
                         objective=s.get("objectivevaluename", "accuracy"),
                         goal=float(s["optimizationgoal"]) if "optimizationgoal" in s else None,
                         request_count=int(s.get("requestcount", 1)),
                         request_number=int(sug.get("requestNumber", 1)),
                         metrics=list(s.get("metricsnames", [])),
                         parameters=[ParameterConfig.from_dict(p) for p in s.get("parameterconfigs", [])],
                         algorithm=sug.get("suggestionAlgorithm", "random"), command=cmd,
                         seed=int(sug.get("seed", 0)))

    @staticmethod
    def from_yaml(path: str) -> "StudySpec":
        with open(path) as f:
            return StudySpec.from_dict(yaml.safe_load(f))


def _command_from_go_template(raw: str) -> list:
    """Extract the container command list from a StudyJob worker Job template (the items before the
    `{{- with .HyperParameters}}` block)."""
    lines = []
    for ln in raw.splitlines():
        if "{{" in ln:
            if not re.sub(r"\{\{-?[^}]*\}\}", "", ln).strip(" -\"'="):
                continue  # hyper-parameter items / control actions: the runner appends name=value itself
            ln = re.sub(r"\{\{-?[^}]*\}\}", "x", ln)
        lines.append(ln)
    doc = "\n".join(lines)
    job = yaml.safe_load(doc) or {}
    try:
        return list(job["spec"]["template"]["spec"]["containers"][0]["command"])
    except (KeyError, IndexError, TypeError):
        return []


class RandomSuggestion:
    def __init__(self, params: list, seed: int = 0):
        self.params, self.rng = params, random.Random(seed)

    def get(self, n: int) -> list[dict]:
        return [{p.name: p.sample(self.rng) for p in self.params} for _ in range(n)]


class GridSuggestion:
    def __init__(self, params: list, points: int = 3):
        self.it = iter(itertools.product(*[[(p.name, v) for v in p.grid(points)] for p in params]))

    def get(self, n: int) -> list[dict]:
        return [dict(x) for x in itertools.islice(self.it, n)]


@dataclass
class Trial:
    trial_id: str
    params: dict
    metrics: dict = field(default_factory=dict)
    status: str = "Created"
    device: str | None = None
    seconds: float = 0.0
    log: str = ""


class StudyRunner:
    """Run a study: `requestcount` rounds of `requestNumber` parallel trials."""

    def __init__(self, spec: StudySpec, trial_fn=None, workdir: str = "/tmp/mifx_hpo", num_gpus: int | None = None,
                 timeout: float | None = None):
        self.spec, self.trial_fn, self.workdir, self.timeout = spec, trial_fn, workdir, timeout
        if num_gpus is None:
            try:
                import torch

                num_gpus = torch.cuda.device_count()
            except Exception:  # noqa: BLE001
                num_gpus = 0
        self.num_gpus = num_gpus
        self.trials: list[Trial] = []
        self.suggest = (GridSuggestion(spec.parameters) if spec.algorithm == "grid"
                        else RandomSuggestion(spec.parameters, spec.seed))
        os.makedirs(workdir, exist_ok=True)

    def _better(self, a: float, b: float) -> bool:
        return a > b if self.spec.optimization == "maximize" else a < b

    def best(self) -> Trial | None:
        done = [t for t in self.trials if self.spec.objective in t.metrics]
        if not done:
            return None
        best = done[0]
        for t in done[1:]:
            if self._better(t.metrics[self.spec.objective], best.metrics[self.spec.objective]):
                best = t
        return best

    def _goal_reached(self) -> bool:
        b = self.best()
        if b is None or self.spec.goal is None:
            return False
        v = b.metrics[self.spec.objective]
        return v >= self.spec.goal if self.spec.optimization == "maximize" else v <= self.spec.goal

    def _run_trial(self, t: Trial) -> Trial:
        t.status, t0 = "Running", time.time()
        names = list(dict.fromkeys(self.spec.metrics + [self.spec.objective]))
        try:
            if self.trial_fn is not None:
                res = self.trial_fn(dict(t.params), t.device)
                t.metrics = {k: float(v) for k, v in res.items()} if isinstance(res, dict) \
                    else {self.spec.objective: float(res)}
            else:
                argv = list(self.spec.command) + [f"{k}={_fmt(v)}" for k, v in t.params.items()]
                env = dict(os.environ)
                if t.device is not None:
                    env["HIP_VISIBLE_DEVICES"] = t.device
                r = subprocess.run(argv, capture_output=True, text=True, env=env, timeout=self.timeout)
                t.log = r.stdout + r.stderr
                t.metrics = parse_metrics(t.log, names)
                if r.returncode != 0:
                    raise RuntimeError(f"worker exited with {r.returncode}")
            t.status = "Succeeded" if self.spec.objective in t.metrics else "MetricsUnavailable"
        except Exception as e:  # noqa: BLE001 - a failed trial does not stop the study
            t.status, t.log = "Failed", (t.log + f"\n{e}").strip()
        t.seconds = time.time() - t0
        return t

    def run(self) -> dict:
        for r in range(self.spec.request_count):
            params = self.suggest.get(self.spec.request_number)
            if not params:
                break
            batch = []
            for i, p in enumerate(params):
                dev = str(len(self.trials) % self.num_gpus) if self.num_gpus else None
                t = Trial(f"{self.spec.name}-{len(self.trials):04d}", p, device=dev)
                self.trials.append(t)
                batch.append(t)
            with cf.ThreadPoolExecutor(max_workers=max(1, min(len(batch), self.num_gpus or len(batch)))) as ex:
                list(ex.map(self._run_trial, batch))
            if self._goal_reached():
                break
        res = self.report()
        with open(os.path.join(self.workdir, f"{self.spec.name}.json"), "w") as f:
            json.dump(res, f, indent=1)
        return res

    def report(self) -> dict:
        b = self.best()
        return {"study": self.spec.name, "objective": self.spec.objective, "optimization": self.spec.optimization,
                "goal_reached": self._goal_reached(),
                "best": None if b is None else {"trial": b.trial_id, "params": b.params, "metrics": b.metrics},
                "trials": [{"trial": t.trial_id, "params": t.params, "metrics": t.metrics, "status": t.status,
                            "device": t.device, "seconds": round(t.seconds, 3)} for t in self.trials]}


def _fmt(v) -> str:
    return f"{v:.6g}" if isinstance(v, float) else str(v)


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(prog="python -m mifx.hpo.study")
    ap.add_argument("spec", nargs="?", help="StudyJob YAML file")
    ap.add_argument("--spec-json", default=None, help="the StudyJob as JSON (the operator's rendered Job)")
    ap.add_argument("--workdir", default="/tmp/mifx_hpo")
    ap.add_argument("--num-gpus", type=int, default=None)
    a = ap.parse_args(argv)
    if (a.spec is None) == (a.spec_json is None):
        ap.error("give a spec file or --spec-json")
    spec = StudySpec.from_yaml(a.spec) if a.spec else StudySpec.from_dict(json.loads(a.spec_json))
    res = StudyRunner(spec, workdir=a.workdir, num_gpus=a.num_gpus).run()
    print(json.dumps(res["best"], indent=1))
    return res


if __name__ == "__main__":
    main()
