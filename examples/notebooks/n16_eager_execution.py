"""Notebook tf2.0/EagerExecution with PyTorch-ROCm eager mode (reference
`notebooks/tf2.0/EagerExecution.ipynb` cells 6-23): eager ops and printing, variables and
in-place updates, gradients, errors surfacing immediately, and the timed 1000x1000 matmul
(the reference's only recorded performance number: 9.87 ms wall on its CPU VM,
`EagerExecution.ipynb:528-530`) on the CPU and on the MI355X (fp32 and bf16 on the MFMA path
through hipBLASLt)."""
from __future__ import annotations

import json
import time

import torch

REFERENCE_CPU_MS = 9.87


def _time(fn, iters: int, sync) -> float:
    fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    sync()
    return (time.perf_counter() - t0) / iters * 1e3


def main(iters: int = 50) -> dict:
    a = torch.tensor([[1.0, 2.0], [3.0, 4.0]])
    print("a + 1 =", a + 1, "\na @ a =", a @ a)               # eager results, no session
    v = torch.zeros(2, requires_grad=False)
    v += torch.tensor([1.0, 2.0])                            # variables are mutable tensors
    w = torch.tensor(3.0, requires_grad=True)
    loss = w * w
    loss.backward()
    print("d(w^2)/dw at 3 =", float(w.grad))                # gradient tape equivalent
    try:
        torch.ones(2, 3) @ torch.ones(2, 3)                  # errors surface at the call site
    except RuntimeError as e:
        print("caught:", str(e).splitlines()[0])

    out = {"reference_cpu_ms": REFERENCE_CPU_MS}
    x = torch.randn(1000, 1000)
    out["cpu_fp32_ms"] = _time(lambda: x @ x, max(3, iters // 5), lambda: None)
    if torch.cuda.is_available():
        xg = x.cuda()
        sync = torch.cuda.synchronize
        out["gpu_fp32_ms"] = _time(lambda: xg @ xg, iters, sync)  # hipBLASLt
        from mifx.ops.gemm import matmul_f32  # the same fp32 op on the hand-written MFMA kernel (edge tiles)

        out["gpu_fp32_hip_ms"] = _time(lambda: matmul_f32(xg, xg), iters, sync)
        out["gpu_fp32_hip_max_abs_err"] = float((matmul_f32(xg, xg) - (x.double() @ x.double()).float().cuda())
                                                .abs().max())
        xb = xg.bfloat16()
        out["gpu_bf16_ms"] = _time(lambda: xb @ xb, iters, sync)
        out["gpu_bf16_tflops"] = 2e9 / (out["gpu_bf16_ms"] * 1e-3) / 1e12
        out["speedup_vs_reference_cpu"] = REFERENCE_CPU_MS / out["gpu_bf16_ms"]
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()
