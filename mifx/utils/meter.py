"""Throughput meter and ROCm trace ranges.

`ExamplesPerSec` reproduces the reference's training-loop log line (`deep_cnn.py:507-538`:
"step N, loss = L (E examples/sec; S sec/batch)") without a host sync on every step: the GPU time
of a window of steps is measured with HIP events. `trace_range(name)` opens a roctx range (via
torch.cuda.nvtx, which maps to roctx on ROCm) so the region shows up in `rocprofv3 --marker-trace`
timelines; it is a no-op on CPU."""
from __future__ import annotations

import contextlib
import time

import torch


class ExamplesPerSec:
    def __init__(self, batch_size: int, every: int = 100, device=None, log=print):
        self.batch, self.every, self.log = batch_size, every, log
        self.cuda = torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self._t0 = None
        self._ev0 = None
        self._n = 0
        self.history: list[dict] = []

    def _now_event(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def start(self) -> None:
        self._n = 0
        if self.cuda:
            self._ev0 = self._now_event()
        self._t0 = time.perf_counter()

    def step(self, step: int, loss=None) -> dict | None:
        """Call once per training step; logs and returns a record every `every` steps."""
        if self._t0 is None:
            self.start()
        self._n += 1
        if self._n < self.every and step != 0:
            return None
        if self.cuda:
            ev1 = self._now_event()
            ev1.synchronize()
            secs = self._ev0.elapsed_time(ev1) / 1e3
        else:
            secs = time.perf_counter() - self._t0
        per_batch = secs / max(1, self._n)
        rec = {"step": step, "examples_per_sec": self.batch / per_batch if per_batch > 0 else float("inf"),
               "sec_per_batch": per_batch}
        if loss is not None:
            rec["loss"] = float(loss.detach()) if torch.is_tensor(loss) else float(loss)
        self.history.append(rec)
        if self.log:
            ls = f", loss = {rec['loss']:.2f}" if "loss" in rec else ""
            self.log(f"step {step}{ls} ({rec['examples_per_sec']:.1f} examples/sec; {per_batch:.3f} sec/batch)")
        self.start()
        return rec


@contextlib.contextmanager
def trace_range(name: str):
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


@contextlib.contextmanager
def heartbeat(label: str, every_s: float = 30.0, stream=None):
    """Print `[label] still running (N s)` every `every_s` seconds while the block runs. First
    training steps can spend minutes inside one call (MIOpen solver search, hipBLASLt tuning, kernel
    JIT); the heartbeat makes such phases visible to whoever watches the log."""
    import sys
    import threading

    out = stream or sys.stderr
    done = threading.Event()
    t0 = time.perf_counter()

    def beat():
        while not done.wait(every_s):
            print(f"[{label}] still running ({time.perf_counter() - t0:.0f} s)", file=out, flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        done.set()
        th.join(timeout=1.0)
