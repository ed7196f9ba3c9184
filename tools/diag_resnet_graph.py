"""ResNetTrainer captured-graph step vs eager step from the same state: where do they differ -- the gradients or the
SGD update? (tests/test_parallel_gpu.py::test_resnet_captured_step_matches_eager)"""
import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402

from mifx.trainer.resnet_trainer import ResNetTrainer, synthetic_imagenet  # noqa: E402

imgs, labels = synthetic_imagenet(48, size=72, classes=10, seed=1)


def make(graph):
    tr = ResNetTrainer(6, "cuda:0", imgs, labels, num_classes=10, lr=0.01, warmup_steps=4, crop=64, seed=5,
                       graph=graph, graph_warmup=2)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    return tr


def rel(a, b):
    num = sum(float((a[k] - b[k]).norm() ** 2) for k in a) ** 0.5
    den = sum(float(b[k].norm() ** 2) for k in b) ** 0.5
    return num / max(den, 1e-30)


trg = make(True)
for _ in range(4):
    trg.step()
ck = {k: v.clone() for k, v in trg.state_dict().items()}
names = [n for n, _ in trg.model.named_parameters()]
p0 = {n: p.detach().float().clone() for n, p in trg.model.named_parameters()}
m0 = {n: trg.opt.state[p]["momentum_buffer"].detach().float().clone() for n, p in trg.model.named_parameters()}
lg = float(trg.step())
gg = {n: p.grad.detach().float().clone() for n, p in trg.model.named_parameters()}
pg = {n: p.detach().float().clone() for n, p in trg.model.named_parameters()}
mg = {n: trg.opt.state[p]["momentum_buffer"].detach().float().clone() for n, p in trg.model.named_parameters()}

tre = make(False)
tre.load_state_dict(ck)
me0 = {n: tre.opt.state[p]["momentum_buffer"].detach().float().clone() for n, p in tre.model.named_parameters()}
le = float(tre.step())
ge = {n: p.grad.detach().float().clone() for n, p in tre.model.named_parameters()}
pe = {n: p.detach().float().clone() for n, p in tre.model.named_parameters()}
me = {n: tre.opt.state[p]["momentum_buffer"].detach().float().clone() for n, p in tre.model.named_parameters()}


def manual(grads, mom0, lr, wd_of):
    out, bufs = {}, {}
    for n in grads:
        d = grads[n] + wd_of(n) * p0[n]
        b = 0.9 * mom0[n] + d
        bufs[n] = b
        out[n] = p0[n] - lr * (d + 0.9 * b)
    return out, bufs


wd = {n: (5e-5 if p.ndim > 1 else 0.0) for n, p in trg.model.named_parameters()}
lr = trg.opt.param_groups[0]["lr"]
exp_g, bg = manual(gg, m0, lr, lambda n: wd[n])
exp_e, be = manual(ge, me0, lr, lambda n: wd[n])
print(json.dumps({"loss_graph": lg, "loss_eager": le, "lr": lr,
                  "momentum_restored_rel": rel(me0, m0),
                  "grad_rel": rel(gg, ge),
                  "update_graph_vs_manual_rel": rel({n: pg[n] - p0[n] for n in names},
                                                    {n: exp_g[n] - p0[n] for n in names}),
                  "update_eager_vs_manual_rel": rel({n: pe[n] - p0[n] for n in names},
                                                    {n: exp_e[n] - p0[n] for n in names}),
                  "momentum_graph_vs_manual_rel": rel(mg, bg), "momentum_eager_vs_manual_rel": rel(me, be),
                  "update_graph_vs_eager_rel": rel({n: pg[n] - p0[n] for n in names},
                                                   {n: pe[n] - p0[n] for n in names})}), flush=True)
worst = sorted(names, key=lambda n: -float((gg[n] - ge[n]).norm() / (ge[n].norm() + 1e-30)))[:6]
print(json.dumps({n: round(float((gg[n] - ge[n]).norm() / (ge[n].norm() + 1e-30)), 5) for n in worst}), flush=True)
