"""Diagnostic: the ResNet-50 DP step forced on one rank (IPC exchange) with a given coalescing threshold
(MIFX_DP_FLUSH_MIN_WG): per-step losses, eager or captured, and the gradients after the first step saved for a diff
across thresholds. usage: python tools/dp_flush_diag.py OUT.pt [--graph] [--batch 256] [--steps 3]"""
import argparse
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    dev = torch.device("cuda", 0)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    imgs, labels = synthetic_imagenet(1024, seed=0, device=dev)
    tr = ResNetTrainer(a.batch, dev, imgs, labels, process_group=torch.distributed.group.WORLD, warmup_steps=10,
                       graph=a.graph, force_dp=True, seed=0)
    losses, grads = [], None
    if os.environ.get("DIAG_STREAMS") == "1":  # which stream the bucket hooks run on, vs the capturing stream
        from mifx.parallel import ddp as ddpm

        orig = ddpm.DataParallel._complete_ready
        seen = set()

        def spy(self):
            s = torch.cuda.current_stream()
            key = (s.cuda_stream, torch.cuda.is_current_stream_capturing())
            if key not in seen:
                seen.add(key)
                print(f"hook stream {s.cuda_stream:#x} capturing={key[1]}", flush=True)
            return orig(self)

        ddpm.DataParallel._complete_ready = spy
        orig_fb = tr._fwd_bwd_captured

        def fb():
            print(f"capture stream {torch.cuda.current_stream().cuda_stream:#x}", flush=True)
            return orig_fb()

        tr._fwd_bwd_captured = fb
    if a.graph and os.environ.get("DIAG_CAPTURE_CHECK") == "1":
        for _ in range(tr.graph_warmup):
            losses.append(float(tr.step()))
        torch.cuda.synchronize()
        before = {n: p.detach().float().cpu().clone() for n, p in tr.model.named_parameters()}
        gb = {n: p.grad.detach().float().cpu().clone() for n, p in tr.model.named_parameters() if p.grad is not None}
        tr._capture()  # capture only: nothing should execute
        torch.cuda.synchronize()
        moved = [n for n, p in tr.model.named_parameters() if not torch.equal(before[n], p.detach().float().cpu())]
        gmoved = [n for n, p in tr.model.named_parameters()
                  if p.grad is not None and n in gb and not torch.equal(gb[n], p.grad.detach().float().cpu())]
        print("weights changed by the capture:", len(moved), moved[:8], "grads changed:", len(gmoved), gmoved[:8],
              flush=True)
    for i in range(a.steps):
        losses.append(float(tr.step()))
        torch.cuda.synchronize()
        if grads is None and (not a.graph or tr._gA is not None):
            grads = {n: p.grad.detach().float().cpu().clone() for n, p in tr.model.named_parameters()
                     if p.grad is not None}
    tr.dp.check()
    torch.save({"losses": losses, "grads": grads, "min_wg": tr.dp.flush_min_wgs, "graph": a.graph}, a.out)
    print(os.environ.get("MIFX_DP_FLUSH_MIN_WG"), a.graph, losses, flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
