"""ResNet-50 v2 inference latency (the serving model, 224 x 224, 1001 classes): the eval-mode network
(bf16 autocast, MIOpen convolutions + BN apply kernels, eager) against the folded form (mifx.models.resnet_infer:
BatchNorms folded into the hand-written convolutions, ReLU in their epilogues), eager and captured in a hipGraph.
CUDA-event timed, one JSON line per batch size.

    python tools/bench_resnet_infer.py [--batches 1 8 32]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.models.resnet import resnet50_v2  # noqa: E402
from mifx.models.resnet_infer import FoldedResNetV2  # noqa: E402


def timeit(fn, it=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 8, 32])
    a = ap.parse_args()
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    m = resnet50_v2(1001).cuda().to(memory_format=torch.channels_last).eval()
    with torch.no_grad():
        f = FoldedResNetV2(m)
        for B in a.batches:
            x = torch.rand(B, 3, 224, 224, device="cuda").contiguous(memory_format=torch.channels_last)

            def eager():
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return m(x)

            t_eager = timeit(eager)
            t_fold = timeit(lambda: f(x))
            run = f.graphed(x)
            t_graph = timeit(lambda: run(x))
            ref = eager().float()
            rel = float((run(x) - ref).norm() / ref.norm())
            print(json.dumps({"batch": B, "ms_eval_model_eager": round(t_eager, 4), "ms_folded_eager": round(t_fold, 4),
                              "ms_folded_hipgraph": round(t_graph, 4),
                              "img_per_s_folded_hipgraph": round(B / t_graph * 1e3, 1),
                              "rel_diff_vs_eval_model": round(rel, 5)}), flush=True)


if __name__ == "__main__":
    main()
