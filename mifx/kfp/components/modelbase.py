"""Typed struct <-> object conversion driven by `__init__` type hints.

Reference behaviour: `sdk/python/kfp/components/modelbase.py:95-287` — a ModelBase subclass is
(de)serialised from/to plain dicts using its constructor signature; `_serialized_names` maps
python attribute names to wire names; Optional/Union/List/Dict/Mapping types are resolved
recursively (Union members tried in order); None-valued attributes are omitted on output."""
from __future__ import annotations

import collections.abc
import inspect
import typing
from typing import Any, Dict, List, Mapping, Union

_NONE = type(None)


def _origin(t):
    return getattr(t, "__origin__", None)


def verify_object_against_type(x, typ) -> bool:
    try:
        parse_object_from_struct_based_on_type(x, typ)
        return True
    except (TypeError, ValueError, KeyError, AttributeError):
        return False


def parse_object_from_struct_based_on_type(struct: Any, typ) -> Any:
    if typ is Any or typ is inspect.Parameter.empty:
        return struct
    if typ is None or typ is _NONE:
        if struct is not None:
            raise TypeError(f"expected None, got {type(struct).__name__}")
        return None
    if isinstance(typ, str):  # forward reference
        raise TypeError(f"unresolved forward reference {typ}")
    if isinstance(typ, type) and issubclass(typ, ModelBase):
        if isinstance(struct, typ):
            return struct
        return typ.from_dict(struct)
    if typ in (str, int, float, bool):
        if typ is float and isinstance(struct, int) and not isinstance(struct, bool):
            return float(struct)
        if not isinstance(struct, typ) or (typ is int and isinstance(struct, bool)):
            raise TypeError(f"expected {typ.__name__}, got {type(struct).__name__}: {struct!r}")
        return struct
    origin = _origin(typ)
    args = getattr(typ, "__args__", ()) or ()
    if origin is Union:
        errors = []
        if struct is None and _NONE in args:
            return None
        for member in args:
            if member is _NONE:
                continue
            try:
                return parse_object_from_struct_based_on_type(struct, member)
            except (TypeError, ValueError, KeyError, AttributeError) as e:
                errors.append(str(e))
        raise TypeError(f"{struct!r} matches none of {args}: {errors}")
    if origin in (list, List, typing.Sequence, collections.abc.Sequence) or typ in (list, List):
        if not isinstance(struct, list):
            raise TypeError(f"expected list, got {type(struct).__name__}")
        et = args[0] if args else Any
        return [parse_object_from_struct_based_on_type(x, et) for x in struct]
    if origin in (dict, Dict, Mapping, typing.Mapping, collections.abc.Mapping) or typ in (dict, Dict):
        if not isinstance(struct, dict):
            raise TypeError(f"expected dict, got {type(struct).__name__}")
        kt, vt = (args + (Any, Any))[:2] if args else (Any, Any)
        return {parse_object_from_struct_based_on_type(k, kt): parse_object_from_struct_based_on_type(v, vt)
                for k, v in struct.items()}
    if isinstance(typ, type) and isinstance(struct, typ):
        return struct
    raise TypeError(f"cannot parse {struct!r} as {typ}")


def _verify(obj, typ) -> None:
    """Checks an already-constructed object (not a wire struct) against a type hint."""
    if typ is Any or typ is inspect.Parameter.empty:
        return
    if typ is None or typ is _NONE:
        if obj is not None:
            raise TypeError(f"expected None, got {type(obj).__name__}")
        return
    if isinstance(typ, type) and issubclass(typ, ModelBase):
        if not isinstance(obj, typ):
            raise TypeError(f"expected {typ.__name__}, got {type(obj).__name__}")
        return
    origin = _origin(typ)
    args = getattr(typ, "__args__", ()) or ()
    if origin is Union:
        for member in args:
            try:
                _verify(obj, member)
                return
            except TypeError:
                continue
        raise TypeError(f"{obj!r} matches none of {args}")
    if origin in (list, List, typing.Sequence, collections.abc.Sequence):
        if not isinstance(obj, list):
            raise TypeError(f"expected list, got {type(obj).__name__}")
        for x in obj:
            _verify(x, args[0] if args else Any)
        return
    if origin in (dict, Dict, Mapping, typing.Mapping, collections.abc.Mapping):
        if not isinstance(obj, dict):
            raise TypeError(f"expected dict, got {type(obj).__name__}")
        kt, vt = (args + (Any, Any))[:2] if args else (Any, Any)
        for k, v in obj.items():
            _verify(k, kt)
            _verify(v, vt)
        return
    parse_object_from_struct_based_on_type(obj, typ)


def convert_object_to_struct(obj, serialized_names: dict | None = None):
    if isinstance(obj, ModelBase):
        return obj.to_dict()
    if isinstance(obj, list):
        return [convert_object_to_struct(x) for x in obj]
    if isinstance(obj, dict):
        return {k: convert_object_to_struct(v) for k, v in obj.items()}
    return obj


class ModelBase:
    _serialized_names: dict = {}

    def __init__(self, args: dict | None = None):
        """Subclasses call `super().__init__(locals())`: every argument is checked against the
        subclass constructor's type hints (TypeError on mismatch) and stored as a field."""
        if args is None:
            return
        _, hints = self._signature()
        fields = {k: v for k, v in args.items() if k != "self" and not k.startswith("_")}
        for k, v in fields.items():
            t = hints.get(k)
            if t is None:
                continue
            try:
                _verify(v, t)
            except (TypeError, ValueError, KeyError, AttributeError) as e:
                raise TypeError(f'Argument for {k} is not compatible with type "{t}": {e}') from None
        self.__dict__.update(fields)

    @classmethod
    def _signature(cls):
        sig = inspect.signature(cls.__init__)
        try:
            hints = typing.get_type_hints(cls.__init__, globalns=vars(__import__(cls.__module__, fromlist=["*"])),
                                          localns={cls.__name__: cls})
        except Exception:  # noqa: BLE001 - fall back to raw annotations
            hints = {}
        params = [p for p in sig.parameters.values() if p.name != "self" and p.kind in
                  (p.POSITIONAL_OR_KEYWORD, p.KEYWORD_ONLY)]
        return params, hints

    @classmethod
    def from_dict(cls, struct: dict):
        if not isinstance(struct, dict):
            raise TypeError(f"{cls.__name__}.from_dict expects a dict, got {type(struct).__name__}")
        params, hints = cls._signature()
        wire_to_attr = {w: a for a, w in cls._serialized_names.items()}
        kwargs = {}
        known = set()
        for wire, value in struct.items():
            attr = wire_to_attr.get(wire, wire)
            p = next((x for x in params if x.name == attr), None)
            if p is None:
                raise KeyError(f"{cls.__name__}: unknown field {wire!r}")
            known.add(attr)
            kwargs[attr] = parse_object_from_struct_based_on_type(value, hints.get(attr, Any))
        for p in params:
            if p.name not in known and p.default is inspect.Parameter.empty:
                raise KeyError(f"{cls.__name__}: missing required field {cls._serialized_names.get(p.name, p.name)!r}")
        return cls(**kwargs)

    def to_dict(self) -> dict:
        params, _ = self._signature()
        out = {}
        for p in params:
            v = getattr(self, p.name, None)
            if v is None:
                continue
            # scalars equal to the constructor default are omitted (reference modelbase.py:178-200)
            if not isinstance(v, (ModelBase, list, dict)) and p.default is not inspect.Parameter.empty \
                    and type(v) is type(p.default) and v == p.default:
                continue
            out[self._serialized_names.get(p.name, p.name)] = convert_object_to_struct(v)
        return out

    def _get_field_names(self):
        return [p.name for p in self._signature()[0]]

    def __eq__(self, other):
        return type(self) is type(other) and self.to_dict() == other.to_dict()

    def __ne__(self, other):
        return not self == other

    def __repr__(self):
        return f"{type(self).__name__}.from_dict({self.to_dict()!r})"
