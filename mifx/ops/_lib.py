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


@functools.lru_cache(maxsize=None)
def load(name: str) -> ctypes.CDLL:
    override = os.environ.get(f"MIFX_LIB_{name.upper()}")  # A/B of diagnostic / variant builds (tools/)
    if override:
        return ctypes.CDLL(override, mode=ctypes.RTLD_GLOBAL)
    path = LIBDIR / f"libmifx_{name}.so"
    if not path.exists():
        if os.environ.get("MIFX_AUTOBUILD", "1") == "1":
            from . import build

            build.build_all(verbose=False)
        if not path.exists():
            raise NativeUnavailable(f"native library {path} is missing; run `python -m mifx.ops.build`")
    return ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)


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
F32 = ctypes.c_float
