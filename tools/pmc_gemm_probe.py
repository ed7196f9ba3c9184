"""The hand-written BERT-base GEMMs at their tuned shapes (4096 tokens), each launched `--reps` times, for a
rocprofv3 --pmc pass (a round-4 GPU batch -> tools/pmc_summary.py): forward NT with the bias(+GELU) epilogue,
input-gradient NT against the transposed weight, weight-gradient TN with its split partials."""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.ops import gemm  # noqa: E402

SHAPES = {"qkv": (768, 2304), "out": (768, 768), "ffn1": (768, 3072), "ffn2": (3072, 768)}  # (in, out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=4096)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda")
    M = a.tokens
    for name, (k, n) in SHAPES.items():
        x = torch.randn(M, k, device=dev, dtype=torch.bfloat16)
        w = (0.02 * torch.randn(n, k, device=dev)).to(torch.bfloat16)
        bias = torch.zeros(n, device=dev, dtype=torch.bfloat16)
        dy = torch.randn(M, n, device=dev, dtype=torch.bfloat16)
        cache = gemm.TransposeCache([w])  # the dX path reads the transposed copy, as in the BERT trainer
        for _ in range(a.reps):
            gemm.linear(x, w, bias)  # routed: the NT kernel where tuned (attention-out), else hipBLASLt
            with gemm.use_transposes(cache):
                gemm._dx(dy, w, None)
            gemm._dw_tensor(dy, x)
        torch.cuda.synchronize()
        print(name, flush=True)


if __name__ == "__main__":
    main()
