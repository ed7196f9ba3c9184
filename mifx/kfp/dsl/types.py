"""DSL parameter types with OpenAPI schema validators and structural type checking.

Reference: `sdk/python/kfp/dsl/types.py:15-166` (Integer, String, Float, Bool, List, Dict, GCSPath,
GCRPath, GCPRegion, GCPProjectID, LocalPath; `check_types`: every property of the upstream
(checked) type must exist with the same value on the downstream (expected) type; an empty type
name matches anything)."""
from __future__ import annotations

import copy


class BaseType:
    """Base of all scalar/artifact types; instances carry their schema as instance attributes so
    that `{TypeName: instance.__dict__}` is the serialized type."""

    _schema: dict | None = None

    def __init__(self):
        if self._schema is not None:
            self.openapi_schema_validator = copy.deepcopy(self._schema)


def _t(name: str, schema: dict):
    return type(name, (BaseType,), {"_schema": schema})


Integer = _t("Integer", {"type": "integer"})
String = _t("String", {"type": "string"})
Float = _t("Float", {"type": "number"})
Bool = _t("Bool", {"type": "boolean"})
List = _t("List", {"type": "array"})
Dict = _t("Dict", {"type": "object"})
GCSPath = _t("GCSPath", {"type": "string", "pattern": "^gs://.*$"})
GCRPath = _t("GCRPath", {"type": "string", "pattern": "^.*gcr\\.io/.*$"})
GCPRegion = _t("GCPRegion", {"type": "string"})
GCPProjectID = _t("GCPProjectID", {"type": "string"})
LocalPath = _t("LocalPath", {"type": "string"})
# AMD additions: typed artifact locations for on-prem MI355X clusters
S3Path = _t("S3Path", {"type": "string", "pattern": "^s3://.*$"})
PVCPath = _t("PVCPath", {"type": "string", "pattern": "^/.*$"})


class InconsistentTypeException(Exception):
    pass


def _instance_to_dict(instance) -> dict:
    return {type(instance).__name__: instance.__dict__}


def _check_valid_type_dict(payload) -> bool:
    if not isinstance(payload, dict) or len(payload) != 1:
        return False
    for name, props in payload.items():
        if not isinstance(props, dict):
            return False
        for pk, pv in props.items():
            if not isinstance(pk, (int, str, float, bool)) or not isinstance(pv, (int, str, float, bool, dict)):
                return False
    return True


def _check_dict_types(checked_type: dict, expected_type: dict) -> bool:
    (cname, cprops), = checked_type.items()
    (ename, eprops), = expected_type.items()
    if cname == "" or ename == "":
        return True
    if cname != ename:
        return False
    for k, v in cprops.items():
        if k not in eprops or eprops[k] != v:
            return False
    return True


def check_types(checked_type, expected_type) -> bool:
    def norm(t):
        if isinstance(t, BaseType):
            return _instance_to_dict(t)
        if isinstance(t, str):
            return {t: {}}
        return t

    return _check_dict_types(norm(checked_type), norm(expected_type))
