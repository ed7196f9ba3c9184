"""Global SDK configuration (reference: `sdk/python/kfp/_config.py:15`).

The user-facing switch is the package attribute `kfp.TYPE_CHECK` (the reference re-exports this module
with `from ._config import *` and its DSL reads `kfp.TYPE_CHECK`, `dsl/_component.py:71`), so
`type_check_enabled()` reads the attribute on the package and `set_type_check()` writes it there."""
import sys

TYPE_CHECK = True


def _root():
    return sys.modules.get("mifx.kfp")


def type_check_enabled() -> bool:
    return bool(getattr(_root(), "TYPE_CHECK", TYPE_CHECK))


def set_type_check(value: bool) -> bool:
    """Sets the switch; returns the previous value."""
    global TYPE_CHECK
    old = type_check_enabled()
    TYPE_CHECK = bool(value)
    root = _root()
    if root is not None:
        root.TYPE_CHECK = bool(value)
    return old
