"""Per-op counters of which path ran: the hand-written gfx950 kernel ("native") or a library / PyTorch fallback.

The hot ops whose native kernels only tile some shapes (the NT / TN GEMMs of mifx.ops.gemm, the fused attention of
mifx.ops.fused_bert) call `count(kind, native)` each time they dispatch, so a run can report how much of a step left
the native path (`snapshot()` after one eager step; graph replays re-run the captured launches without Python, so
the counts of the captured step are the counts of every replayed step)."""
from __future__ import annotations

import threading

_LOCK = threading.Lock()
_C: dict[str, list[int]] = {}


def count(kind: str, native: bool) -> None:
    with _LOCK:
        c = _C.setdefault(kind, [0, 0])
        c[0 if native else 1] += 1


def reset() -> None:
    with _LOCK:
        _C.clear()


def snapshot() -> dict[str, dict[str, int]]:
    """{kind: {"native": n, "fallback": m}}."""
    with _LOCK:
        return {k: {"native": v[0], "fallback": v[1]} for k, v in sorted(_C.items())}


def fallback_fraction() -> float:
    with _LOCK:
        n = sum(v[0] + v[1] for v in _C.values())
        return sum(v[1] for v in _C.values()) / n if n else 0.0
