"""Run one weight-gradient GEMM shape on the TN kernel (and hipBLASLt) repeatedly: a target for rocprofv3 --pmc.
`python tools/tn_probe.py [M N T cfg splits]`"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mifx.ops import gemm  # noqa: E402

M, N, T, cfg, s = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (3072, 768, 4096, 0, 1)))
dy = torch.randn(T, M, device="cuda").to(torch.bfloat16)
x = torch.randn(T, N, device="cuda").to(torch.bfloat16)
for _ in range(20):
    gemm.gemm_tn(dy, x, cfg, s)
for _ in range(5):
    dy.t() @ x
torch.cuda.synchronize()
print("done")
