"""ctypes loader for the in-tree native libraries built by :mod:`mifx.ops.build`.

Policy: on a machine with a visible GPU the HIP libraries are REQUIRED — a missing or stale
library raises instead of silently falling back to PyTorch, so GPU tests prove the native path
ran. On a CPU-only host callers may use the documented PyTorch reference implementations.
"""
from __future__ import annotations

import ctypes
import functools
import os
from pathlib import Path

import torch  # noqa: F401  (must load torch's libamdhip64 before our libraries bind to it)

LIBDIR = Path(__file__).resolve().parent / "lib"


class NativeUnavailable(RuntimeError):
    pass


def gpu_available() -> bool:
    return torch.cuda.is_available()


def _source_of(name: str):
    from . import build

    for ext in (".hip", ".cpp"):
        p = build.CSRC / f"{name}{ext}"
        if p.exists():
            return p
    return None


@functools.lru_cache(maxsize=None)
def load(name: str) -> ctypes.CDLL:
    """Load libmifx_<name>.so. The library must report the hash of the sources next to it (mifx_src_hash,
    compiled in by mifx.ops.build): a stale or foreign binary is rebuilt (MIFX_AUTOBUILD=1, the default) or
    refused -- never silently run."""
    from . import build

    override = os.environ.get(f"MIFX_LIB_{name.upper()}")  # A/B of diagnostic / variant builds (tools/)
    if override:
        return ctypes.CDLL(override, mode=ctypes.RTLD_GLOBAL)
    path = LIBDIR / f"libmifx_{name}.so"
    src = _source_of(name)
    want = build.source_hash(src) if src is not None else None
    stale = not path.exists() or (want is not None and build.embedded_hash(path) != want)
    if stale and os.environ.get("MIFX_AUTOBUILD", "1") == "1":
        build.build_all(verbose=False)
        stale = not path.exists() or (want is not None and build.embedded_hash(path) != want)
    if not path.exists():
        raise NativeUnavailable(f"native library {path} is missing; run `python -m mifx.ops.build`")
    if stale:
        raise NativeUnavailable(f"native library {path} was not built from the current {src.name} "
                                f"(hash {build.embedded_hash(path)} != {want}); run `python -m mifx.ops.build`")
    lib = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
    if want is not None:
        f = lib.mifx_src_hash
        f.restype = ctypes.c_char_p
        got = f().decode()
        if got != want:
            raise NativeUnavailable(f"{path}: loaded library reports source hash {got}, sources are {want}")
    return lib


def available(name: str) -> bool:
    try:
        load(name)
        return True
    except (NativeUnavailable, OSError):
        return False


def stream_handle(device: torch.device | None = None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: torch.Tensor | None) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with HIP error code {rc}")


def sig(lib: ctypes.CDLL, fname: str, argtypes: list, restype=ctypes.c_int):
    f = getattr(lib, fname)
    f.argtypes = argtypes
    f.restype = restype
    return f


VP = ctypes.c_void_p
I32 = ctypes.c_int
I64 = ctypes.c_longlong
U64 = ctypes.c_ulonglong
F32 = ctypes.c_float
