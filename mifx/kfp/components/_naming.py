"""Name sanitisation / uniquing helpers (reference: `sdk/python/kfp/components/_naming.py:33-101`)."""
from __future__ import annotations

import hashlib
import re
import time
from typing import Callable, Mapping, Sequence


def _normalize_identifier_name(name: str) -> str:
    n = name.lower()
    n = re.sub(r"[\W_]", " ", n)
    n = re.sub(" +", " ", n).strip()
    if re.match(r"\d", n):
        n = "n" + n
    return n


def _sanitize_kubernetes_resource_name(name: str) -> str:
    return _normalize_identifier_name(name).replace(" ", "-")


def _sanitize_python_function_name(name: str) -> str:
    return _normalize_identifier_name(name).replace(" ", "_")


def _sanitize_file_name(name: str) -> str:
    return re.sub("[^-_.0-9a-zA-Z]+", "_", name)


def _convert_to_human_name(name: str) -> str:
    return name.replace("_", " ").replace("-", " ").strip().capitalize()


def _generate_unique_suffix(data) -> str:
    return hashlib.sha256(str((data, time.time())).encode()).hexdigest()[:8]


def _make_name_unique_by_adding_index(name: str, collection, delimiter: str) -> str:
    unique, i = name, 2
    while unique in collection:
        unique = f"{name}{delimiter}{i}"
        i += 1
    return unique


def _convert_name_and_make_it_unique_by_adding_number(name: str, used, conversion_func: Callable[[str], str]) -> str:
    conv = conversion_func(name)
    i = 2
    while conv in used:
        conv = conversion_func(f"{name} {i}")
        i += 1
    return conv


def generate_unique_name_conversion_table(names: Sequence[str], conversion_func: Callable[[str], str]
                                          ) -> Mapping[str, str]:
    fwd, rev = {}, {}
    for n in names:
        if n in fwd:
            raise ValueError(f"Original name {n} is not unique.")
        c = _convert_name_and_make_it_unique_by_adding_number(n, rev, conversion_func)
        fwd[n] = c
        rev[c] = n
    return fwd
