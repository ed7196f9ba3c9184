"""PipelineParam: a future value passed between ops, serialisable inline in strings.

Reference: `sdk/python/kfp/dsl/_pipeline_param.py:22-242` — serialized form
``{{pipelineparam:op=<op>;name=<name>;value=<value>}}`` (``;type=<type>;`` appended when typed),
recursive extraction from strings / lists / dicts / k8s models, comparison operators building
``ConditionOperator`` tuples, k8s name sanitisation."""
from __future__ import annotations

import re
from collections import namedtuple

from ._metadata import TypeMeta

ConditionOperator = namedtuple("ConditionOperator", "operator operand1 operand2")
PipelineParamTuple = namedtuple("PipelineParamTuple", "name op value type pattern")


def sanitize_k8s_name(name: str) -> str:
    return re.sub("-+", "-", re.sub("[^-0-9a-z]+", "-", name.lower())).lstrip("-").rstrip("-")


_RE_TYPED = re.compile(r"{{pipelineparam:op=([\w\s_-]*);name=([\w\s_-]+);value=(.*?);type=(.*?);}}")
_RE_PLAIN = re.compile(r"{{pipelineparam:op=([\w\s_-]*);name=([\w\s_-]+);value=(.*?)}}")


def match_serialized_pipelineparam(payload: str) -> list[PipelineParamTuple]:
    out = []
    typed = _RE_TYPED.findall(payload)
    if typed:
        for op, name, value, typ in typed:
            out.append(PipelineParamTuple(sanitize_k8s_name(name), sanitize_k8s_name(op), value, typ,
                                          "{{pipelineparam:op=%s;name=%s;value=%s;type=%s;}}" % (op, name, value, typ)))
        return out
    for op, name, value in _RE_PLAIN.findall(payload):
        out.append(PipelineParamTuple(sanitize_k8s_name(name), sanitize_k8s_name(op), value, "",
                                      "{{pipelineparam:op=%s;name=%s;value=%s}}" % (op, name, value)))
    return out


def _extract_pipelineparams(payloads) -> list["PipelineParam"]:
    if isinstance(payloads, str):
        payloads = [payloads]
    tuples = []
    for p in payloads:
        tuples += match_serialized_pipelineparam(p)
    return [PipelineParam(t.name, t.op, t.value, TypeMeta.deserialize(t.type), pattern=t.pattern)
            for t in dict.fromkeys(tuples)]


def extract_pipelineparams_from_any(payload) -> list["PipelineParam"]:
    if not payload:
        return []
    if isinstance(payload, PipelineParam):
        return [payload]
    if isinstance(payload, str):
        return list(dict.fromkeys(_extract_pipelineparams(payload)))
    items = None
    if isinstance(payload, (list, tuple)):
        items = payload
    elif isinstance(payload, dict):
        items = list(payload.values())
    elif isinstance(getattr(payload, "swagger_types", None), dict):
        items = [getattr(payload, k) for k in payload.swagger_types]
    elif isinstance(getattr(payload, "openapi_types", None), dict):
        items = [getattr(payload, k) for k in payload.openapi_types]
    if items is None:
        return []
    out = []
    for it in items:
        out += extract_pipelineparams_from_any(it)
    return list(dict.fromkeys(out))


class PipelineParam:
    """A parameter of a pipeline or an output of an op.

    `op_name` is the producing op (None for pipeline arguments); `value` is an immediate value."""

    def __init__(self, name: str, op_name: str | None = None, value=None, param_type: TypeMeta | None = None,
                 pattern: str | None = None):
        valid = r"^[A-Za-z][A-Za-z0-9\s_-]*$"
        if not re.match(valid, name):
            raise ValueError(f"Only letters, numbers, spaces, '_', and '-' are allowed in name. Must begin with letter: "
                             f"{name}")
        if op_name and value:
            raise ValueError("op_name and value cannot be both set.")
        self.name = name
        self.op_name = op_name if op_name else None
        self.value = value if value else None
        self.param_type = param_type or TypeMeta()
        # serialized form at creation time: survives later name sanitisation so the compiler can
        # still find (and replace) this param inside strings built before compilation
        self.pattern = pattern or str(self)

    @property
    def full_name(self) -> str:
        return f"{self.op_name}-{self.name}" if self.op_name else self.name

    def __str__(self) -> str:
        op = self.op_name or ""
        val = self.value if self.value else ""
        if self.param_type is None:
            return "{{pipelineparam:op=%s;name=%s;value=%s}}" % (op, self.name, val)
        return "{{pipelineparam:op=%s;name=%s;value=%s;type=%s;}}" % (op, self.name, val,
                                                                      self.param_type.serialize())

    def __repr__(self):
        return str({type(self).__name__: self.__dict__})

    def __eq__(self, other):
        return ConditionOperator("==", self, other)

    def __ne__(self, other):
        return ConditionOperator("!=", self, other)

    def __lt__(self, other):
        return ConditionOperator("<", self, other)

    def __le__(self, other):
        return ConditionOperator("<=", self, other)

    def __gt__(self, other):
        return ConditionOperator(">", self, other)

    def __ge__(self, other):
        return ConditionOperator(">=", self, other)

    def __hash__(self):
        return hash((self.op_name, self.name))

    def ignore_type(self):
        """Drops the type so type checking passes for this argument (chainable)."""
        self.param_type = TypeMeta()
        return self
