"""Artifacts and channels of the TFX-style component model.

Reference: TFX 0.13 artifact/channel contract used by `airflow-dags/taxi_pipeline.py:68-132`
(``component.outputs.examples``, ``csv_input(path)``) and the MLMD type names of
`notebooks/tfx_utils.py:28-47`.
"""
from __future__ import annotations

import json
from typing import Any, Iterable

from ..metadata.proto import Artifact as MlmdArtifact
from ..metadata.proto import ArtifactType, STRING, INT


class Artifact:
    """A typed, URI-addressed pipeline artifact (one per split for example-like outputs)."""

    TYPE_NAME = "Artifact"
    PROPERTIES = {"type_name": STRING, "split": STRING, "name": STRING, "state": STRING, "span": INT}

    def __init__(self, type_name: str | None = None, split: str = "", uri: str = ""):
        self.type_name = type_name or self.TYPE_NAME
        self.uri = uri
        self.split = split
        self.id: int | None = None
        self.type_id: int | None = None
        self.name = ""
        self.producer_component = ""
        self.state = ""
        self.custom_properties: dict[str, Any] = {}

    # ---- MLMD mapping ------------------------------------------------------------------------
    def mlmd_type(self) -> ArtifactType:
        return ArtifactType(name=self.type_name, properties=dict(self.PROPERTIES))

    def to_mlmd(self) -> MlmdArtifact:
        a = MlmdArtifact(type_id=self.type_id, uri=self.uri, id=self.id)
        a.properties["type_name"] = self.type_name
        a.properties["split"] = self.split
        a.properties["name"] = self.name
        a.properties["state"] = self.state or "published"
        for k, v in self.custom_properties.items():
            a.custom_properties[k] = v
        return a

    @classmethod
    def from_mlmd(cls, a: MlmdArtifact, type_name: str) -> "Artifact":
        o = cls(type_name=type_name, split=a.properties["split"].string_value or "", uri=a.uri)
        o.id, o.type_id = a.id, a.type_id
        o.name = a.properties["name"].string_value or ""
        o.state = a.properties["state"].string_value or ""
        o.custom_properties = {k: v.value for k, v in a.custom_properties.items()}
        return o

    def to_json(self) -> dict:
        return {"type_name": self.type_name, "uri": self.uri, "split": self.split, "id": self.id,
                "name": self.name, "custom_properties": self.custom_properties}

    @classmethod
    def from_json(cls, d: dict) -> "Artifact":
        o = cls(d["type_name"], d.get("split", ""), d.get("uri", ""))
        o.id = d.get("id")
        o.name = d.get("name", "")
        o.custom_properties = dict(d.get("custom_properties", {}))
        return o

    def __repr__(self):
        return f"Artifact({self.type_name}, split={self.split!r}, uri={self.uri!r}, id={self.id})"


class Channel:
    """A typed stream of artifacts connecting a producer output to consumer inputs."""

    def __init__(self, type_name: str, artifacts: Iterable[Artifact] | None = None):
        self.type_name = type_name
        self._artifacts = list(artifacts or [])
        self.producer = None  # (component, output key)

    def get(self) -> list[Artifact]:
        return list(self._artifacts)

    def set(self, artifacts: Iterable[Artifact]) -> None:
        arts = list(artifacts)
        for a in arts:
            if a.type_name != self.type_name:
                raise TypeError(f"channel of {self.type_name} got {a.type_name}")
        self._artifacts = arts

    def __repr__(self):
        p = f" from {self.producer[0].id}.{self.producer[1]}" if self.producer else ""
        return f"Channel({self.type_name}{p}, {len(self._artifacts)} artifacts)"


class ChannelMap(dict):
    """dict of channels with attribute access (``component.outputs.examples``)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def get_all(self) -> dict:
        return dict(self)


# ---- TFX 0.13 artifact type names (notebooks/tfx_utils.py:28-47) ----------------------------
EXTERNAL = "ExternalPath"
EXAMPLES = "ExamplesPath"
EXAMPLE_STATS = "ExampleStatisticsPath"
SCHEMA = "SchemaPath"
EXAMPLE_VALIDATION = "ExampleValidationPath"
TRANSFORM = "TransformPath"
MODEL = "ModelExportPath"
MODEL_EVAL = "ModelEvalPath"
MODEL_BLESSING = "ModelBlessingPath"
PUSHED_MODEL = "ModelPushPath"


def external_input(uri: str) -> Channel:
    a = Artifact(EXTERNAL, uri=uri)
    return Channel(EXTERNAL, [a])


def csv_input(uri: str) -> Channel:
    """`tfx.utils.dsl_utils.csv_input` equivalent (taxi_pipeline.py:70)."""
    return external_input(uri)


def dumps_artifacts(d: dict[str, list[Artifact]]) -> str:
    return json.dumps({k: [a.to_json() for a in v] for k, v in d.items()})


def loads_artifacts(s: str) -> dict[str, list[Artifact]]:
    return {k: [Artifact.from_json(x) for x in v] for k, v in json.loads(s).items()}
