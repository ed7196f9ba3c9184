"""Inference graphs: A/B tests, multi-armed bandits, outlier detection (Seldon-Core-style serving).

The reference vendors Seldon Core prototypes (`install-kubeflow/ks_app/vendor/kubeflow/seldon/
prototypes/{abtest,mab,outlier-detector,serve-simple}-v1alpha2.jsonnet`): a SeldonDeployment whose
predictor `graph` is a tree of nodes typed MODEL / ROUTER / TRANSFORMER / COMBINER, e.g.
`RANDOM_ABTEST(ratioA)` over two classifiers, an epsilon-greedy router (`n_branches`, `epsilon`,
`verbose`) that learns from `/feedback` rewards, or a Mahalanobis outlier-detector TRANSFORMER in
front of a model. This module executes such a graph in-process (one Python server, models on the
GPU) and exposes Seldon's REST protocol:

    POST /api/v0.1/predictions  {"data": {"ndarray": [[...], ...]}}
        -> {"data": {"names": [...], "ndarray": [...]}, "meta": {"routing": {...}, "tags": {...}}}
    POST /api/v0.1/feedback     {"request": ..., "response": <with meta.routing>, "reward": r}

Graph specs are the same dicts the prototypes emit (`graph: {name, type, implementation,
parameters: [{name, value, type}], children: [...]}`); MODEL nodes resolve by name to a callable
or a mifx SavedModel export directory."""

import math
import threading
from typing import Callable

import numpy as np
import torch

_CASTS = {"FLOAT": float, "DOUBLE": float, "INT": int, "BOOL": lambda v: str(v).lower() in ("1", "true", "yes"),
          "STRING": str}


def _params(spec: dict) -> dict:
    return {p["name"]: _CASTS.get(p.get("type", "STRING"), str)(p["value"]) for p in spec.get("parameters", []) or []}


class Node:
    def __init__(self, name: str, children: list | None = None):
        self.name, self.children = name, children or []

    def predict(self, x: np.ndarray, meta: dict) -> np.ndarray:
        raise NotImplementedError

    def feedback(self, reward: float, routing: dict) -> None:
        for c in self.children:
            c.feedback(reward, routing)

    def walk(self):
        yield self
        for c in self.children:
            yield from c.walk()


class ModelNode(Node):
    """Leaf model: a callable ndarray -> ndarray, or a mifx SavedModel directory (GPU if present)."""

    def __init__(self, name: str, model):
        super().__init__(name)
        if isinstance(model, str):
            from .saved_model import load

            loaded = load(model)
            self.fn = lambda x: np.asarray(loaded.predict(x.tolist())["predictions"])
        else:
            self.fn = model

    def predict(self, x, meta):
        return np.asarray(self.fn(x))


class RandomABTest(Node):
    """RANDOM_ABTEST: route each request to child 0 with probability ratioA, else child 1."""

    def __init__(self, name: str, children: list, ratioA: float = 0.5, seed: int | None = None):
        super().__init__(name, children)
        if len(children) != 2:
            raise ValueError("RANDOM_ABTEST needs exactly two children")
        self.ratio = float(ratioA)
        self.rng = np.random.default_rng(seed)
        self._lock = threading.Lock()

    def route(self, x) -> int:
        with self._lock:
            return 0 if self.rng.random() < self.ratio else 1

    def predict(self, x, meta):
        b = self.route(x)
        meta.setdefault("routing", {})[self.name] = b
        return self.children[b].predict(x, meta)


class EpsilonGreedy(Node):
    """Epsilon-greedy multi-armed bandit router (seldonio/mab_epsilon_greedy): exploit the branch with
    the best observed mean reward with probability 1-epsilon, explore uniformly otherwise. Rewards
    arrive through feedback() with the routing the response carried."""

    def __init__(self, name: str, children: list, n_branches: int | None = None, epsilon: float = 0.1,
                 verbose: bool = False, seed: int | None = None):
        super().__init__(name, children)
        self.n = int(n_branches or len(children))
        if self.n != len(children):
            raise ValueError(f"n_branches={self.n} but {len(children)} children")
        self.epsilon, self.verbose = float(epsilon), bool(verbose)
        self.tries = np.zeros(self.n)
        self.successes = np.zeros(self.n)
        self.best = 0
        self.rng = np.random.default_rng(seed)
        self._lock = threading.Lock()

    def route(self, x) -> int:
        with self._lock:
            if self.rng.random() < self.epsilon:
                return int(self.rng.integers(self.n))
            return self.best

    def predict(self, x, meta):
        b = self.route(x)
        meta.setdefault("routing", {})[self.name] = b
        return self.children[b].predict(x, meta)

    def feedback(self, reward: float, routing: dict) -> None:
        b = routing.get(self.name)
        if b is not None:
            with self._lock:
                self.tries[b] += 1
                self.successes[b] += float(reward)
                rates = np.where(self.tries > 0, self.successes / np.maximum(self.tries, 1), 0.0)
                self.best = int(np.argmax(rates))
            if self.verbose:
                print(f"{self.name}: branch {b} reward {reward}; best branch {self.best} rates {rates.round(3)}")
            self.children[b].feedback(reward, routing)


class MahalanobisOutlier(Node):
    """Online Mahalanobis-distance outlier detector TRANSFORMER (seldonio/outlier_mahalanobis): keeps a
    running mean/covariance of the features seen (Welford, fp64 on the device), scores each row
    against the statistics BEFORE the batch is absorbed, tags `outlier-score` / `is-outlier`
    (score > threshold) in the response meta and forwards the input unchanged to its child."""

    def __init__(self, name: str, children: list, threshold: float = 25.0, n_stdev: float | None = None,
                 start_clip: int = 50, max_n: int = -1, device=None):
        super().__init__(name, children)
        self.threshold = float(threshold if n_stdev is None else n_stdev ** 2)
        self.start = int(start_clip)
        self.max_n = int(max_n)
        self.dev = torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))
        self.n = 0
        self.mean = None
        self.m2 = None
        self._lock = threading.Lock()

    def score(self, x: np.ndarray) -> np.ndarray:
        t = torch.as_tensor(np.asarray(x, np.float64), device=self.dev).reshape(len(x), -1)
        with self._lock:
            if self.n < 2:
                s = torch.zeros(len(t), dtype=torch.float64, device=self.dev)
            else:
                cov = self.m2 / (self.n - 1) + 1e-6 * torch.eye(t.shape[1], dtype=torch.float64, device=self.dev)
                d = t - self.mean
                s = (d @ torch.linalg.solve(cov, d.T)).diagonal()
            for row in t:  # Welford update, row order (deterministic)
                if self.max_n > 0 and self.n >= self.max_n:
                    break
                if self.mean is None:
                    self.mean = torch.zeros_like(row)
                    self.m2 = torch.zeros(row.numel(), row.numel(), dtype=torch.float64, device=self.dev)
                self.n += 1
                delta = row - self.mean
                self.mean += delta / self.n
                self.m2 += torch.outer(delta, row - self.mean)
        return s.cpu().numpy()

    def predict(self, x, meta):
        s = self.score(x)
        warm = self.n > self.start
        meta.setdefault("tags", {})["outlier-score"] = s.tolist()
        meta["tags"]["is-outlier"] = [bool(v > self.threshold) and warm for v in s]
        return self.children[0].predict(x, meta) if self.children else np.asarray(x)


class AverageCombiner(Node):
    def predict(self, x, meta):
        return np.mean([np.asarray(c.predict(x, meta), np.float64) for c in self.children], axis=0)


_IMPLS = {"RANDOM_ABTEST": RandomABTest, "EPSILON_GREEDY": EpsilonGreedy, "AVERAGE_COMBINER": AverageCombiner,
          "MAHALANOBIS_OUTLIER": MahalanobisOutlier}
_BY_NAME = {"eg-router": EpsilonGreedy, "outlier-detector": MahalanobisOutlier}


def build_graph(spec: dict, models: dict[str, Callable | str], seed: int | None = None) -> Node:
    """Build the executable tree of a predictor `graph` spec. MODEL nodes look up `models[name]`."""
    children = [build_graph(c, models, seed) for c in spec.get("children", []) or []]
    kind = spec.get("type", "MODEL")
    impl = spec.get("implementation")
    params = _params(spec)
    name = spec["name"]
    if impl in _IMPLS or name in _BY_NAME:
        cls = _IMPLS.get(impl) or _BY_NAME[name]
        extra = {"seed": seed} if cls in (RandomABTest, EpsilonGreedy) else {}
        return cls(name, children, **params, **extra)
    if kind == "MODEL":
        if name not in models:
            raise KeyError(f"no model registered for graph node {name!r}")
        return ModelNode(name, models[name])
    if kind == "COMBINER":
        return AverageCombiner(name, children)
    raise ValueError(f"unsupported graph node {name!r} (type {kind}, implementation {impl})")


def predictor_graph(deployment: dict) -> dict:
    """The first predictor's graph of a SeldonDeployment manifest (or the graph itself)."""
    if "graph" in deployment:
        return deployment["graph"]
    return deployment["spec"]["predictors"][0]["graph"]


class GraphServer:
    def __init__(self, root: Node, names: list[str] | None = None):
        self.root, self.names = root, names
        self.requests = 0

    def _decode(self, msg: dict) -> np.ndarray:
        d = msg.get("data", msg)
        if "ndarray" in d:
            return np.asarray(d["ndarray"], np.float64)
        if "tensor" in d:
            return np.asarray(d["tensor"]["values"], np.float64).reshape(d["tensor"]["shape"])
        raise ValueError("request needs data.ndarray or data.tensor")

    def predict(self, msg: dict) -> dict:
        x = self._decode(msg)
        meta: dict = {}
        y = np.asarray(self.root.predict(x, meta))
        self.requests += 1
        names = self.names or [f"t:{i}" for i in range(y.shape[-1] if y.ndim > 1 else 1)]
        out = {"data": {"names": names, "ndarray": y.tolist()}, "meta": meta}
        return out

    def feedback(self, msg: dict) -> dict:
        routing = ((msg.get("response") or {}).get("meta") or {}).get("routing") or {}
        reward = float(msg.get("reward", 0.0))
        if not math.isfinite(reward):
            raise ValueError("reward must be finite")
        self.root.feedback(reward, routing)
        return {"meta": {"routing": routing}}


def create_app(server: GraphServer):
    from fastapi import FastAPI, HTTPException, Request

    app = FastAPI(title="mifx inference graph")

    @app.post("/api/v0.1/predictions")
    async def predictions(req: Request):
        try:
            return server.predict(await req.json())
        except (ValueError, KeyError) as e:
            raise HTTPException(400, str(e)) from e

    @app.post("/api/v0.1/feedback")
    async def feedback(req: Request):
        try:
            return server.feedback(await req.json())
        except (ValueError, KeyError) as e:
            raise HTTPException(400, str(e)) from e

    @app.get("/ping")
    def ping():
        return "pong"

    return app
