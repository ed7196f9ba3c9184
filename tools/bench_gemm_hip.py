"""Hand-written MFMA GEMM (csrc/gemm.hip) vs hipBLASLt (torch F.linear) on BERT-base's forward projection shapes
(B=32, S=128: M = 4096 tokens), random bf16 operands; every tile configuration that tiles the shape. For FFN-in
also the fused bias + GELU epilogue against F.linear + the unfused bias_gelu kernel. CUDA-event timing of 50
back-to-back calls after 10 warmups. One JSON line per measurement."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))

from mifx.ops import fused_bert as fb  # noqa: E402
from mifx.ops import gemm  # noqa: E402

M = 4096
SHAPES = {"qkv": (768, 2304), "out": (768, 768), "ffn1": (768, 3072), "ffn2": (3072, 768)}


def timeit(fn, iters=50):
    for _ in range(10):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters  # us


def main():
    torch.manual_seed(0)
    dev = "cuda"
    cfgs = gemm.config_details()
    # --dx: the backward's input-gradient products dX[M, in] = dY[M, out] . W[out, in], run as NT products against a
    # transposed weight copy (W^T [in, out], K-contiguous) vs the library's dY @ W (what the backward runs today)
    dx = "--dx" in sys.argv
    shapes = {nm: (n, k) for nm, (k, n) in SHAPES.items()} if dx else SHAPES
    for name, (k, n) in shapes.items():
        x = (torch.rand(M, k, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device=dev) * 2 - 1) * k ** -0.5).to(torch.bfloat16)
        b = (torch.rand(n, device=dev) * 0.2 - 0.1).to(torch.bfloat16)
        flop = 2.0 * M * k * n
        if dx:
            wt = w.t().contiguous()  # [k, n]: the layer's weight [out = k, in = n]
            rows = [("hipblaslt dY @ W (NN)", lambda: x @ wt), ("transpose W (per step)", lambda: w.t().contiguous())]
            name = name + "_dx"
        else:
            rows = [("hipblaslt F.linear(x, w)", lambda: F.linear(x, w)),
                    ("hipblaslt F.linear(x, w, b)", lambda: F.linear(x, w, b))]
        if name == "ffn1":
            rows.append(("hipblaslt F.linear + bias_gelu kernel", lambda: fb.bias_gelu(F.linear(x, w), b)))
        for i, (bm, bn, opt) in enumerate(cfgs):
            if M % bm or n % bn or k % 64:
                continue
            tag = f"hip cfg{i} {bm}x{bn} opt{opt}"
            rows.append((f"{tag} none", lambda i=i: gemm.gemm_nt(x, w, None, 0, cfg=i)))
            if dx:
                continue
            rows.append((f"{tag} +bias", lambda i=i: gemm.gemm_nt(x, w, b, 1, cfg=i)))
            if name == "ffn1":
                rows.append((f"{tag} +bias+gelu (y and z)", lambda i=i: gemm.gemm_nt(x, w, b, 2, cfg=i)))
        if dx:  # the NN kernel on dY [M, k] x W [k, n] (no transposed copy)
            for i, (bm, bn, ns) in enumerate(gemm.nn_configs()):
                if M % bm or n % bn or k % 64:
                    continue
                rows.append((f"nn cfg{i} {bm}x{bn} ring{ns}", lambda i=i: gemm.gemm_nn(x, wt, None, cfg=i)))
                rows.append((f"nn cfg{i} {bm}x{bn} ring{ns} +R", lambda i=i: gemm.gemm_nn(x, wt, rr, cfg=i)))
            rr = torch.randn(M, n, device=dev).to(torch.bfloat16)
            rows.append(("hipblaslt addmm(R, dY, W)", lambda: torch.addmm(rr, x, wt)))
        for label, fn in rows:
            us = timeit(fn)
            print(json.dumps({"gemm": name, "M": M, "N": n, "K": k, "impl": label, "us": round(us, 2),
                              "tflops": round(flop / us / 1e6, 1)}), flush=True)
    print(json.dumps({"auto_pick": {nm: gemm.pick_config(M, n, k) for nm, (k, n) in SHAPES.items()}}), flush=True)


if __name__ == "__main__":
    main()
