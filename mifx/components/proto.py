"""Argument messages of the TFX 0.13 components (trainer_pb2 / evaluator_pb2 / pusher_pb2
equivalents used in `airflow-dags/taxi_pipeline.py:97-120`)."""
from __future__ import annotations

from dataclasses import asdict, dataclass, field


class _Msg:
    def to_dict(self) -> dict:
        return asdict(self)


@dataclass
class TrainArgs(_Msg):
    num_steps: int = 0
    splits: list = field(default_factory=lambda: ["train"])


@dataclass
class EvalArgs(_Msg):
    num_steps: int = 0
    splits: list = field(default_factory=lambda: ["eval"])


@dataclass
class SingleSlicingSpec(_Msg):
    column_for_slicing: list = field(default_factory=list)  # [] = overall slice; 2 cols = feature cross


@dataclass
class FeatureSlicingSpec(_Msg):
    specs: list = field(default_factory=list)  # list[SingleSlicingSpec]

    def to_dict(self) -> dict:
        return {"specs": [s.to_dict() if isinstance(s, SingleSlicingSpec) else s for s in self.specs]}


@dataclass
class Filesystem(_Msg):
    base_directory: str = ""


@dataclass
class PushDestination(_Msg):
    filesystem: Filesystem = field(default_factory=Filesystem)
    Filesystem = Filesystem  # pusher_pb2.PushDestination.Filesystem

    def to_dict(self) -> dict:
        return {"filesystem": {"base_directory": self.filesystem.base_directory}}


@dataclass
class SplitConfig(_Msg):
    """ExampleGen output split: name + hash buckets (TFX default train:eval = 2:1)."""
    name: str = "train"
    hash_buckets: int = 2


def default_splits() -> list[SplitConfig]:
    return [SplitConfig("train", 2), SplitConfig("eval", 1)]


def from_dict(cls, d):
    if d is None or isinstance(d, cls):
        return d
    if cls is FeatureSlicingSpec:
        return FeatureSlicingSpec([SingleSlicingSpec(**s) if isinstance(s, dict) else s for s in d.get("specs", [])])
    if cls is PushDestination:
        return PushDestination(Filesystem(**d.get("filesystem", {})))
    return cls(**d)
