"""ML-Metadata-compatible record types (the subset of `ml_metadata.proto.metadata_store_pb2`
the reference uses: `notebooks/utils.py:28-48,64-85,237-244,272-318`, `notebooks/tfx_utils.py:53-65`).

Plain dataclasses instead of protobuf messages; field and enum names match MLMD so code written
against `metadata_store_pb2` reads naturally (``event.type == Event.OUTPUT``,
``artifact.properties['split'].string_value``)."""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from typing import Union


class PropertyType(enum.IntEnum):
    UNKNOWN = 0
    INT = 1
    DOUBLE = 2
    STRING = 3


INT, DOUBLE, STRING = PropertyType.INT, PropertyType.DOUBLE, PropertyType.STRING


@dataclass
class Value:
    int_value: int | None = None
    double_value: float | None = None
    string_value: str | None = None

    @staticmethod
    def of(v: Union[int, float, str, "Value"]) -> "Value":
        if isinstance(v, Value):
            return v
        if isinstance(v, bool):
            return Value(int_value=int(v))
        if isinstance(v, int):
            return Value(int_value=v)
        if isinstance(v, float):
            return Value(double_value=v)
        return Value(string_value=str(v))

    def WhichOneof(self, _name: str = "value") -> str | None:  # noqa: N802 (protobuf API)
        for k in ("int_value", "double_value", "string_value"):
            if getattr(self, k) is not None:
                return k
        return None

    @property
    def value(self):
        k = self.WhichOneof()
        return getattr(self, k) if k else None


class _Props(dict):
    """dict[str, Value] that auto-wraps raw Python values on assignment."""

    def __setitem__(self, k, v):
        super().__setitem__(k, Value.of(v))

    def __missing__(self, k):  # protobuf map semantics: reading creates an empty Value
        v = Value()
        super().__setitem__(k, v)
        return v


def _props(d=None) -> _Props:
    p = _Props()
    for k, v in (d or {}).items():
        p[k] = v
    return p


@dataclass
class ArtifactType:
    name: str
    properties: dict = field(default_factory=dict)  # name -> PropertyType
    id: int | None = None


@dataclass
class ExecutionType:
    name: str
    properties: dict = field(default_factory=dict)
    id: int | None = None


@dataclass
class ContextType:
    name: str
    properties: dict = field(default_factory=dict)
    id: int | None = None


class ArtifactState(enum.IntEnum):
    UNKNOWN = 0
    PENDING = 1
    LIVE = 2
    MARKED_FOR_DELETION = 3
    DELETED = 4


class ExecutionState(enum.IntEnum):
    UNKNOWN = 0
    NEW = 1
    RUNNING = 2
    COMPLETE = 3
    FAILED = 4
    CACHED = 5
    CANCELED = 6


@dataclass
class Artifact:
    type_id: int | None = None
    uri: str = ""
    properties: _Props = field(default_factory=_props)
    custom_properties: _Props = field(default_factory=_props)
    id: int | None = None
    name: str | None = None
    state: ArtifactState = ArtifactState.UNKNOWN
    create_time_since_epoch: int = 0
    last_update_time_since_epoch: int = 0

    def __post_init__(self):
        if not isinstance(self.properties, _Props):
            self.properties = _props(self.properties)
        if not isinstance(self.custom_properties, _Props):
            self.custom_properties = _props(self.custom_properties)


@dataclass
class Execution:
    type_id: int | None = None
    properties: _Props = field(default_factory=_props)
    custom_properties: _Props = field(default_factory=_props)
    id: int | None = None
    name: str | None = None
    last_known_state: ExecutionState = ExecutionState.UNKNOWN
    create_time_since_epoch: int = 0
    last_update_time_since_epoch: int = 0

    def __post_init__(self):
        if not isinstance(self.properties, _Props):
            self.properties = _props(self.properties)
        if not isinstance(self.custom_properties, _Props):
            self.custom_properties = _props(self.custom_properties)


@dataclass
class Context:
    type_id: int | None = None
    name: str = ""
    properties: _Props = field(default_factory=_props)
    custom_properties: _Props = field(default_factory=_props)
    id: int | None = None

    def __post_init__(self):
        if not isinstance(self.properties, _Props):
            self.properties = _props(self.properties)
        if not isinstance(self.custom_properties, _Props):
            self.custom_properties = _props(self.custom_properties)


@dataclass
class EventPathStep:
    index: int | None = None
    key: str | None = None


@dataclass
class Event:
    class Type(enum.IntEnum):
        UNKNOWN = 0
        DECLARED_OUTPUT = 1
        DECLARED_INPUT = 2
        INPUT = 3
        OUTPUT = 4
        INTERNAL_INPUT = 5
        INTERNAL_OUTPUT = 6

    artifact_id: int | None = None
    execution_id: int | None = None
    type: "Event.Type" = 0
    path: list = field(default_factory=list)  # list[EventPathStep]
    milliseconds_since_epoch: int = 0


# MLMD-style class-level enum aliases: Event.OUTPUT, Event.INPUT, ...
for _m in Event.Type:
    setattr(Event, _m.name, _m)


def is_output_event(e: Event) -> bool:
    return e.type in (Event.Type.DECLARED_OUTPUT, Event.Type.OUTPUT)


def is_input_event(e: Event) -> bool:
    return e.type in (Event.Type.DECLARED_INPUT, Event.Type.INPUT)


@dataclass
class SqliteMetadataSourceConfig:
    filename_uri: str = ""
    connection_mode: int = 3  # READWRITE_OPENCREATE

    READONLY = 1
    READWRITE = 2
    READWRITE_OPENCREATE = 3


@dataclass
class ConnectionConfig:
    sqlite: SqliteMetadataSourceConfig = field(default_factory=SqliteMetadataSourceConfig)
    fake_database: bool = False  # in-memory store
