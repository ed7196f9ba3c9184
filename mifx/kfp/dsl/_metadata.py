"""Type / parameter / component / pipeline metadata extracted from function signatures.

Reference: `sdk/python/kfp/dsl/_metadata.py:19-250`."""
from __future__ import annotations

import inspect
import json

import yaml

from .types import BaseType, _check_valid_type_dict, _instance_to_dict


class BaseMeta:
    def to_dict(self):
        raise NotImplementedError

    def serialize(self) -> str:
        return yaml.dump(self.to_dict())

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__


class TypeMeta(BaseMeta):
    def __init__(self, name: str = "", properties: dict | None = None):
        self.name = name
        self.properties = {} if properties is None else properties

    def to_dict_or_str(self):
        return self.name if not self.properties else {self.name: self.properties}

    @staticmethod
    def from_dict_or_str(payload) -> "TypeMeta":
        t = TypeMeta()
        if isinstance(payload, dict):
            if not _check_valid_type_dict(payload):
                raise ValueError(f"{payload} is not a valid type dict")
            (t.name, props), = payload.items()
            t.properties = dict(props)
        elif isinstance(payload, str):
            t.name = payload
        else:
            raise ValueError("from_dict_or_str expects a dict or str")
        return t

    def serialize(self) -> str:
        return str(self.to_dict_or_str())

    @staticmethod
    def deserialize(payload) -> "TypeMeta":
        if isinstance(payload, str) and payload.startswith("{"):
            import ast

            try:
                payload = ast.literal_eval(payload)
            except (ValueError, SyntaxError):
                pass
        return TypeMeta.from_dict_or_str(payload)


class ParameterMeta(BaseMeta):
    def __init__(self, name: str, description: str = "", param_type: TypeMeta | None = None, default=None):
        self.name = name
        self.description = description
        self.param_type = TypeMeta() if param_type is None else param_type
        self.default = default

    def to_dict(self):
        return {"name": self.name, "description": self.description, "type": self.param_type.to_dict_or_str(),
                "default": self.default}


class ComponentMeta(BaseMeta):
    def __init__(self, name: str, description: str = "", inputs=None, outputs=None):
        self.name = name
        self.description = description
        self.inputs = [] if inputs is None else inputs
        self.outputs = [] if outputs is None else outputs

    def to_dict(self):
        return {"name": self.name, "description": self.description, "inputs": [i.to_dict() for i in self.inputs],
                "outputs": [o.to_dict() for o in self.outputs]}


class PipelineMeta(BaseMeta):
    def __init__(self, name: str, description: str = "", inputs=None):
        self.name = name
        self.description = description
        self.inputs = [] if inputs is None else inputs

    def to_dict(self):
        return {"name": self.name, "description": self.description, "inputs": [i.to_dict() for i in self.inputs]}


def _annotation_to_typemeta(annotation) -> TypeMeta:
    if isinstance(annotation, BaseType):
        return TypeMeta.deserialize(_instance_to_dict(annotation))
    if isinstance(annotation, type) and issubclass(annotation, BaseType):
        return TypeMeta.deserialize(_instance_to_dict(annotation()))
    if isinstance(annotation, str):
        return TypeMeta.deserialize(annotation)
    if isinstance(annotation, dict):
        if not _check_valid_type_dict(annotation):
            raise ValueError(f"Annotation {annotation} is not a valid type dictionary.")
        return TypeMeta.deserialize(annotation)
    return TypeMeta()


def _defaults(spec) -> dict:
    out = {}
    if spec.defaults:
        for arg, d in zip(reversed(spec.args), reversed(spec.defaults)):
            out[arg] = d
    return out


def _extract_component_metadata(func) -> ComponentMeta:
    from ._pipeline_param import PipelineParam

    spec = inspect.getfullargspec(func)
    defaults = _defaults(spec)
    inputs = []
    for arg in spec.args:
        d = defaults.get(arg)
        if isinstance(d, PipelineParam):
            d = d.value
        t = _annotation_to_typemeta(spec.annotations[arg]) if arg in spec.annotations else TypeMeta()
        inputs.append(ParameterMeta(name=arg, param_type=t, default=d))
    outputs = []
    if "return" in spec.annotations and isinstance(spec.annotations["return"], dict):
        for name, ann in spec.annotations["return"].items():
            outputs.append(ParameterMeta(name=name, param_type=_annotation_to_typemeta(ann)))
    return ComponentMeta(name=func.__name__, inputs=inputs, outputs=outputs)


def _extract_pipeline_metadata(func, validate: bool = True) -> PipelineMeta:
    """Pipeline signature -> PipelineMeta; with `validate`, defaults are checked against any
    `openapi_schema_validator` in their type (done at compile time, not at decoration)."""
    from ._pipeline_param import PipelineParam

    spec = inspect.getfullargspec(func)
    defaults = _defaults(spec)
    meta = PipelineMeta(name=getattr(func, "_pipeline_name", func.__name__),
                        description=getattr(func, "_pipeline_description", func.__doc__))
    for arg in spec.args:
        d = defaults.get(arg)
        if isinstance(d, PipelineParam):
            d = d.value
        t = _annotation_to_typemeta(spec.annotations[arg]) if arg in spec.annotations else TypeMeta()
        schema = t.properties.get("openapi_schema_validator")
        if validate and schema is not None and d is not None:
            _validate_schema(d, json.loads(schema) if isinstance(schema, str) else schema)
        meta.inputs.append(ParameterMeta(name=arg, param_type=t, default=d))
    return meta


def _validate_schema(value, schema: dict) -> None:
    """Small OpenAPI/JSON-schema validator (type + pattern), jsonschema-free."""
    import re

    kinds = {"integer": int, "string": str, "number": (int, float), "boolean": bool, "array": list, "object": dict}
    t = schema.get("type")
    if t in kinds and not isinstance(value, kinds[t]):
        raise ValueError(f"{value!r} is not of type {t}")
    if "pattern" in schema and isinstance(value, str) and not re.search(schema["pattern"], value):
        raise ValueError(f"{value!r} does not match {schema['pattern']}")
