"""bf16 GEMM throughput (torch.matmul -> hipBLASLt) on BERT-base's training shapes (B=32, S=128: M=4096 tokens),
forward / data-gradient / weight-gradient layouts, TFLOP/s. Peak dense bf16 on MI355X is ~2.5 PFLOP/s."""
import json
import time

import torch

M = 4096
SHAPES = {"qkv": (768, 2304), "out": (768, 768), "ffn1": (768, 3072), "ffn2": (3072, 768)}


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    dev = "cuda"
    for name, (k, n) in SHAPES.items():
        x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)  # nn.Linear weight [out, in]
        dy = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * k * n
        for kind, fn in (("fwd x@w.T", lambda: x @ w.t()), ("dgrad dy@w", lambda: dy @ w),
                         ("wgrad dy.T@x", lambda: dy.t() @ x)):
            t = timeit(fn)
            print(json.dumps({"gemm": name, "kind": kind, "us": round(t * 1e6, 1),
                              "tflops": round(flop / t / 1e12, 1)}), flush=True)


if __name__ == "__main__" and __import__("sys").argv[1:] == []:
    main()


def splitk():
    """weight-gradient as split-K: S batched [n x M/S] @ [M/S x k] GEMMs (fp32 out) + a sum over S."""
    dev = "cuda"
    for name, (k, n) in SHAPES.items():
        x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
        flop = 2.0 * M * k * n
        for S in (2, 4, 8, 16):
            xs = x.view(S, M // S, k)
            dys = dy.view(S, M // S, n).transpose(1, 2)

            def fn():
                return torch.bmm(dys, xs).sum(0)
            t = timeit(fn)
            print(json.dumps({"gemm": name, "kind": f"wgrad split-K bmm S={S} + sum", "us": round(t * 1e6, 1),
                              "tflops": round(flop / t / 1e12, 1)}), flush=True)


if __name__ == "__main__" and __import__("sys").argv[1:] == ["splitk"]:
    splitk()

