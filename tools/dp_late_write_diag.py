"""Diagnostic: does anything write a data-parallel bucket after its exchange was launched? ResNet-50 forced one-rank
DP, eager steps with the exchange joined right after each launch (MIFX_DP_COMM=join: with one rank the exchange
returns its input, so a late write survives); each bucket's contents are snapshotted at launch and compared with the
final gradients after finish(). Prints the parameters whose bucket slot changed after launch."""
import os
import socket
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIFX_DP_COMM", "join")


def main():
    from mifx.parallel import ddp as ddpm
    from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet

    dev = torch.device("cuda", 0)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    torch.distributed.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    imgs, labels = synthetic_imagenet(1024, seed=0, device=dev)
    tr = ResNetTrainer(int(os.environ.get("DIAG_BATCH", "256")), dev, imgs, labels,
                       process_group=torch.distributed.group.WORLD, warmup_steps=10, graph=False, force_dp=True)
    snaps = {}
    orig = ddpm.DataParallel._launch

    def spy(self, b):
        snaps[id(b)] = b.buf.clone()
        return orig(self, b)

    ddpm.DataParallel._launch = spy
    names = {id(p): n for n, p in tr.model.named_parameters()}
    orig_finish = ddpm.DataParallel.finish
    report = []

    def finish_spy(self):
        orig_finish(self)  # (the comparison runs before the optimizer, which may update gradients in place)
        torch.cuda.synchronize()
        late = []
        for bi, b in enumerate(self.buckets):
            s = snaps.get(id(b))
            if s is None:
                continue
            for pi, p in enumerate(b.params):
                off = b.offsets[pi]
                a, c = s[off:off + p.numel()], b.buf[off:off + p.numel()]
                if not torch.equal(a, c):
                    late.append((bi, names[id(p)], float((a - c).abs().max())))
        report.append((len(snaps), late))

    ddpm.DataParallel.finish = finish_spy
    for step in range(3):
        snaps.clear()
        report.clear()
        tr.step()
        torch.cuda.synchronize()
        n, late = report[-1]
        print(f"step {step}: buckets {len(tr.dp.buckets)} launched {n}, slots written after launch: {late[:20]}",
              flush=True)
    torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
