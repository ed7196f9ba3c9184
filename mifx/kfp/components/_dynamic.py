"""Create a python function with an explicit signature that forwards its arguments as a dict.

Reference: `sdk/python/kfp/components/_dynamic.py:20-68` (task factories get a real signature:
required inputs first, defaults preserved)."""
from __future__ import annotations

import functools
import inspect
from typing import Callable, Sequence


class KwParameter(inspect.Parameter):
    def __init__(self, name, default=inspect.Parameter.empty, annotation=inspect.Parameter.empty):
        super().__init__(name, inspect.Parameter.POSITIONAL_OR_KEYWORD, default=default, annotation=annotation)


def create_function_from_parameters(func: Callable[[dict], object], parameters: Sequence[inspect.Parameter],
                                    documentation: str | None = None, func_name: str | None = None,
                                    func_filename: str | None = None) -> Callable:
    sig = inspect.Signature(parameters)

    def f(*args, **kwargs):
        bound = sig.bind(*args, **kwargs)
        bound.apply_defaults()
        return func(dict(bound.arguments))

    f.__signature__ = sig
    f.__name__ = func_name or "f"
    f.__qualname__ = f.__name__
    f.__doc__ = documentation
    if func_filename:
        f.__module__ = func_filename
    return f


_ = functools
