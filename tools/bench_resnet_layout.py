"""ResNet-50 training step time: channels_last vs contiguous (NCHW), bf16 autocast, with MIOpen find."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.models.resnet import resnet50_v2  # noqa: E402


def run(fmt, B=256, steps=10, warm=5):
    torch.manual_seed(0)
    m = resnet50_v2(1000).cuda().to(memory_format=fmt)
    opt = torch.optim.SGD(m.parameters(), lr=0.1, momentum=0.9)
    x = torch.randn(B, 3, 224, 224, device="cuda").to(memory_format=fmt)
    y = torch.randint(0, 1000, (B,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        opt.step()

    for _ in range(warm):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    return {"format": str(fmt), "ms_per_step": dt * 1e3, "images_per_sec": B / dt}


if __name__ == "__main__":
    torch.backends.cudnn.benchmark = True
    for fmt in (torch.contiguous_format, torch.channels_last):
        print(json.dumps(run(fmt)), flush=True)
