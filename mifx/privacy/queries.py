"""Private-query protocol: clip / accumulate / noise / normalise over nested tensor records.

Reference: `optimizers/private_queries.py:26-130` (PrivateQuery with initial_global_state,
derive_sample_params, initial_sample_state, accumulate_record, get_query_result; Sum/Average
specialisations), `gaussian_query.py:31-198`, `nested_query.py:30-123`, `no_privacy_query.py:27-95`.

Records are arbitrary nests (list / tuple / dict) of torch tensors. For the single-pass GPU path the
DP optimizer bypasses per-record accumulation and hands all microbatch gradients at once to
`GaussianSumQuery.aggregate_batch` (-> the fused HIP clip/sum/noise kernel)."""
from __future__ import annotations

import abc
import collections
import math

import torch

# ---- tiny nest utilities ---------------------------------------------------------------------


def nest_flatten(x) -> list:
    if isinstance(x, dict):
        return [leaf for k in sorted(x) for leaf in nest_flatten(x[k])]
    if isinstance(x, (list, tuple)) and not hasattr(x, "_fields"):
        return [leaf for v in x for leaf in nest_flatten(v)]
    return [x]


def nest_pack(template, leaves: list):
    it = iter(leaves)

    def rec(t):
        if isinstance(t, dict):
            return {k: rec(t[k]) for k in sorted(t)}
        if isinstance(t, (list, tuple)) and not hasattr(t, "_fields"):
            return type(t)(rec(v) for v in t)
        return next(it)

    out = rec(template)
    return out


def nest_map(fn, *nests):
    flats = [nest_flatten(n) for n in nests]
    return nest_pack(nests[0], [fn(*xs) for xs in zip(*flats)])


def _map_up_to(shallow, fn, *nests):
    """Apply fn at the leaves of `shallow` (a query structure); deeper structure of `nests` is passed whole."""
    if isinstance(shallow, dict):
        return {k: _map_up_to(shallow[k], fn, *[n[k] for n in nests]) for k in shallow}
    if isinstance(shallow, (list, tuple)) and not hasattr(shallow, "_fields"):
        if any(not isinstance(n, (list, tuple)) or len(n) != len(shallow) for n in nests):
            raise ValueError("record structure is incompatible with the query structure")
        return type(shallow)(_map_up_to(s, fn, *[n[i] for n in nests]) for i, s in enumerate(shallow))
    return fn(shallow, *nests)


# ---- protocol --------------------------------------------------------------------------------


class PrivateQuery(abc.ABC):
    def initial_global_state(self):
        return ()

    def derive_sample_params(self, global_state):
        return ()

    @abc.abstractmethod
    def initial_sample_state(self, global_state, template):
        ...

    @abc.abstractmethod
    def accumulate_record(self, params, sample_state, record):
        ...

    @abc.abstractmethod
    def get_query_result(self, sample_state, global_state):
        ...


class PrivateSumQuery(PrivateQuery):
    def get_query_result(self, sample_state, global_state):
        return self.get_noised_sum(sample_state, global_state)

    @abc.abstractmethod
    def get_noised_sum(self, sample_state, global_state):
        ...


class PrivateAverageQuery(PrivateQuery):
    def get_query_result(self, sample_state, global_state):
        return self.get_noised_average(sample_state, global_state)

    @abc.abstractmethod
    def get_noised_average(self, sample_state, global_state):
        ...


def clip_by_global_norm(tensors: list, clip: float):
    norm = math.sqrt(sum(float(t.double().pow(2).sum()) for t in tensors))
    scale = clip / norm if norm > clip else 1.0
    return [t * scale for t in tensors], norm


class GaussianSumQuery(PrivateSumQuery):
    """Clip each record to global L2 norm `l2_norm_clip`, sum, add N(0, stddev^2)."""

    GlobalState = collections.namedtuple("GlobalState", ["l2_norm_clip", "stddev"])

    def __init__(self, l2_norm_clip: float, stddev: float, generator: torch.Generator | None = None):
        self._clip, self._stddev = float(l2_norm_clip), float(stddev)
        self._gen = generator

    def initial_global_state(self):
        return self.GlobalState(self._clip, self._stddev)

    def derive_sample_params(self, global_state):
        return global_state.l2_norm_clip

    def initial_sample_state(self, global_state, template):
        return nest_map(torch.zeros_like, template)

    def accumulate_record(self, params, sample_state, record):
        clipped, _ = clip_by_global_norm(nest_flatten(record), params)
        return nest_map(torch.add, sample_state, nest_pack(record, clipped))

    def get_noised_sum(self, sample_state, global_state):
        def add_noise(v):
            if global_state.stddev == 0:
                return v
            return v + global_state.stddev * torch.randn(v.shape, generator=self._gen, dtype=v.dtype).to(v.device)

        return nest_map(add_noise, sample_state), global_state

    def aggregate_batch(self, G: torch.Tensor, global_state, denominator: float = 1.0, seed: int = 0,
                        offset: int = 0) -> torch.Tensor:
        """All microbatch records at once: G [M, P] -> noised (sum / denominator) [P] (fused HIP kernel on GPU)."""
        from ..ops.dp import clip_sum_noise

        return clip_sum_noise(G, global_state.l2_norm_clip, global_state.stddev, denominator, seed, offset)


class GaussianAverageQuery(PrivateAverageQuery):
    """GaussianSumQuery followed by division by a fixed `denominator`."""

    GlobalState = collections.namedtuple("GlobalState", ["sum_state", "denominator"])

    def __init__(self, l2_norm_clip: float, sum_stddev: float, denominator: float,
                 generator: torch.Generator | None = None):
        self._numerator = GaussianSumQuery(l2_norm_clip, sum_stddev, generator)
        self._denominator = float(denominator)

    def initial_global_state(self):
        return self.GlobalState(self._numerator.initial_global_state(), self._denominator)

    def derive_sample_params(self, global_state):
        return self._numerator.derive_sample_params(global_state.sum_state)

    def initial_sample_state(self, global_state, template):
        return self._numerator.initial_sample_state(global_state.sum_state, template)

    def accumulate_record(self, params, sample_state, record):
        return self._numerator.accumulate_record(params, sample_state, record)

    def get_noised_average(self, sample_state, global_state):
        s, new_sum = self._numerator.get_noised_sum(sample_state, global_state.sum_state)
        return nest_map(lambda v: v / global_state.denominator, s), self.GlobalState(new_sum, global_state.denominator)

    def aggregate_batch(self, G, global_state, seed: int = 0, offset: int = 0):
        return self._numerator.aggregate_batch(G, global_state.sum_state, global_state.denominator, seed, offset)


class NoPrivacySumQuery(PrivateSumQuery):
    """Exact sum (baseline)."""

    def initial_sample_state(self, global_state, template):
        return nest_map(torch.zeros_like, template)

    def accumulate_record(self, params, sample_state, record):
        return nest_map(torch.add, sample_state, record)

    def get_noised_sum(self, sample_state, global_state):
        return sample_state, global_state


class NoPrivacyAverageQuery(PrivateAverageQuery):
    """Exact (optionally weighted) average (baseline)."""

    def initial_sample_state(self, global_state, template):
        return nest_map(torch.zeros_like, template), 0.0

    def accumulate_record(self, params, sample_state, record, weight: float = 1.0):
        s, d = sample_state
        return nest_map(lambda a, b: a + weight * b, s, record), d + weight

    def get_noised_average(self, sample_state, global_state):
        s, d = sample_state
        return nest_map(lambda v: v / d, s), global_state


class NestedQuery(PrivateQuery):
    """A nest of queries applied to the matching sub-structures of each record."""

    def __init__(self, queries):
        self._queries = queries

    def _each(self, method: str, *args):
        return _map_up_to(self._queries, lambda q, *a: getattr(q, method)(*a), *args)

    def initial_global_state(self):
        return _map_up_to(self._queries, lambda q: q.initial_global_state())

    def derive_sample_params(self, global_state):
        return self._each("derive_sample_params", global_state)

    def initial_sample_state(self, global_state, template):
        return self._each("initial_sample_state", global_state, template)

    def accumulate_record(self, params, sample_state, record):
        return self._each("accumulate_record", params, sample_state, record)

    def get_query_result(self, sample_state, global_state):
        pairs = self._each("get_query_result", sample_state, global_state)
        results = _map_up_to(self._queries, lambda q, p: p[0], pairs)
        states = _map_up_to(self._queries, lambda q, p: p[1], pairs)
        return results, states
