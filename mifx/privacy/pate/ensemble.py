"""All PATE teachers trained at once: the ensemble as ONE grouped network.

The reference trains the `nb_teachers` teachers one after another (`research/pate_2017/train_teachers.py:44-96`,
one process per `--teacher_id`, each a 3000-step run of a small CNN on a 60000/nb_teachers-example shard) and
then restores them one by one to label the student data (`train_student.py:53-84`). That is hundreds of
launch-bound little trainings. MI355X-first, the teachers become one network whose convolutions are grouped
convolutions (group t = teacher t), whose dense layers are batched matmuls over the teacher dimension and
whose LRN normalises each teacher's channel block on its own; every shard sits in HBM at once, interleaved as
the channel dimension of one NHWC batch, so a single step advances every teacher on its own batch
(SURVEY §2.10 "ensemble / partitioned-data parallel"). Across GPUs, rank r trains teachers r, r+W, ...
with no communication.

Equivalence: teacher t of the ensemble follows exactly the recipe of `deep_cnn.train` on shard t — same
initial weights (the sequential trainer seeds every teacher identically), same batches
(`batch_indices`), same staircase-decayed SGD and EMA (one fused multi-tensor kernel for the whole
ensemble) — and writes the same per-teacher checkpoint files, so `deep_cnn.softmax_preds` and the student
pipeline read them unchanged. `tests/test_pate_training.py` checks the ensemble against the sequential
trainer teacher by teacher."""
from __future__ import annotations

import math
import time
from datetime import datetime

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ...models.cnn import _same_pad, same_maxpool
from ...ops import cnn_ops, gconv, pool
from . import deep_cnn


USE_HIP_CONV = True  # csrc/gconv.hip for the eligible stride-1 layers (False: F.conv2d, for A/B and exact tests)


def _conv_specs(model: nn.Module):
    """(name, stride) of the conv layers of a PateCNN in forward order."""
    if model.deeper:
        return [(f"convs.{i}", c.stride[0]) for i, c in enumerate(model.convs)]
    return [("c1", 1), ("c2", 1)]


def _fc_names(model: nn.Module):
    return ["f1", "out"] if model.deeper else ["f3", "f4", "out"]


class PateEnsemble(nn.Module):
    """`T` copies of a `PateCNN` evaluated as one grouped network. Input: [B, T*Cin, H, W] (teacher t's image in
    channels [t*Cin, (t+1)*Cin)); output logits [T, B, classes]."""

    def __init__(self, template: nn.Module, T: int):
        super().__init__()
        if template.dropout:
            raise ValueError("the teacher ensemble trains without dropout (deep_cnn.train's teacher default)")
        self.T, self.deeper = int(T), template.deeper
        self.conv_specs = _conv_specs(template)
        self.fc_names = _fc_names(template)
        sd = {k: v.detach() for k, v in template.state_dict().items()}
        self.conv_w = nn.ParameterList()
        self.conv_b = nn.ParameterList()
        for name, _ in self.conv_specs:
            self.conv_w.append(nn.Parameter(sd[f"{name}.weight"].repeat(T, 1, 1, 1).clone()))
            self.conv_b.append(nn.Parameter(sd[f"{name}.bias"].repeat(T).clone()))
        self.fc_w = nn.ParameterList()
        self.fc_b = nn.ParameterList()
        for name in self.fc_names:  # [T, in, out] / [T, 1, out] for baddbmm
            self.fc_w.append(nn.Parameter(sd[f"{name}.weight"].t().unsqueeze(0).repeat(T, 1, 1).contiguous()))
            self.fc_b.append(nn.Parameter(sd[f"{name}.bias"].view(1, 1, -1).repeat(T, 1, 1).contiguous()))
        self.kernels = [template.get_submodule(n).kernel_size[0] for n, _ in self.conv_specs]

    # -------------------------------------------------------------------------------- forward
    @property
    def col_input(self) -> bool:
        """First layer as a 1x1 grouped GEMM over an im2col image (Cin * k * k <= 32 taps padded to 32 channels per
        teacher): the Cin = 1 layer has no 32-channel reduction of its own, and the image of the resident dataset is
        built once (`conv_input`), not per step."""
        w = self.conv_w[0]
        return (USE_HIP_CONV and self.conv_specs[0][1] == 1 and self.kernels[0] % 2 == 1
                and w.shape[1] * self.kernels[0] ** 2 <= 32)

    def conv_input(self, x: torch.Tensor, chunk: int = 256) -> torch.Tensor:
        """[n, T*Cin, H, W] images -> [n, T*32, H, W] SAME-padded im2col image (channels-last storage; bf16 on the
        GPU), channel t*32 + (c*k + r)*k + s = x[t*Cin + c] at offset (r - k//2, s - k//2), zero-padded to 32."""
        if not self.col_input:
            return x
        n, TC, H, W = x.shape
        k, T = self.kernels[0], self.T
        cin, p = TC // T, self.kernels[0] // 2
        dt = torch.bfloat16 if x.is_cuda else x.dtype
        out = torch.empty(n, H, W, T, 32, device=x.device, dtype=dt)
        for i in range(0, n, chunk):
            xb = F.pad(x[i:i + chunk].to(dt), (p, p, p, p))
            cols = xb.unfold(2, k, 1).unfold(3, k, 1)  # [b, T*Cin, H, W, k, k]
            b = cols.shape[0]
            cols = cols.reshape(b, T, cin, H, W, k * k).permute(0, 3, 4, 1, 2, 5).reshape(b, H, W, T, cin * k * k)
            out[i:i + chunk, ..., :cin * k * k] = cols
            out[i:i + chunk, ..., cin * k * k:] = 0
        t = out.view(n, H, W, T * 32).permute(0, 3, 1, 2)
        return t if x.is_cuda else t.contiguous()

    def _conv0_col(self, xcol: torch.Tensor, relu: bool = False) -> torch.Tensor:
        w = self.conv_w[0]
        taps = w.shape[1] * self.kernels[0] ** 2
        wc = F.pad(w.reshape(w.shape[0], taps), (0, 32 - taps)).view(w.shape[0], 32, 1, 1)
        return gconv.conv2d(xcol, wc, self.conv_b[0], padding=0, groups=self.T, relu=relu)

    def _conv(self, i: int, x: torch.Tensor, relu: bool = False) -> torch.Tensor:
        k, s = self.kernels[i], self.conv_specs[i][1]
        if USE_HIP_CONV and s == 1 and k % 2 == 1:  # SAME = symmetric pad k//2: grouped MFMA conv when eligible
            return gconv.conv2d(x, self.conv_w[i], self.conv_b[i], padding=k // 2, groups=self.T, relu=relu)
        if USE_HIP_CONV and x.is_cuda:  # strided SAME: explicit (asymmetric) pad, then the strided kernel
            return gconv.conv2d(_same_pad(x, k, s), self.conv_w[i], self.conv_b[i], padding=0, groups=self.T,
                                relu=relu, stride=s)
        # (weights in the activations' dtype: the HIP layers hand bf16 activations on even outside autocast)
        y = F.conv2d(_same_pad(x, k, s), self.conv_w[i].to(x.dtype), self.conv_b[i].to(x.dtype), stride=s,
                     groups=self.T)
        return F.relu(y) if relu else y

    def _lrn(self, y: torch.Tensor) -> torch.Tensor:
        """tf.nn.lrn(4, 1, 0.001/9, 0.75) over each teacher's own channel block: the NHWC rows of every
        (pixel, teacher) pair are one [C]-row of the HIP LRN kernel."""
        B, TC, h, w = y.shape
        C = TC // self.T
        v = y.permute(0, 2, 3, 1).reshape(B * h * w * self.T, C, 1, 1)
        if not v.is_contiguous(memory_format=torch.channels_last):
            v = v.contiguous()
        out = cnn_ops.lrn(v, depth_radius=4, bias=1.0, alpha=0.001 / 9.0, beta=0.75)
        return out.reshape(B, h, w, TC).permute(0, 3, 1, 2)

    def forward(self, x: torch.Tensor, col: bool = False) -> torch.Tensor:
        """`col=True`: x is `conv_input(images)` (the first layer runs as a 1x1 grouped GEMM)."""
        if not self.deeper:
            y = self._conv0_col(x) if col else self._conv(0, x)
            p = pool.max_pool3s2_same(y, relu=True)  # relu + SAME max-pool in one HIP pass each way
            y = self._lrn(p if p is not None else same_maxpool(F.relu(y), 3, 2))
            y = self._conv(1, y, relu=True)
            y = same_maxpool(self._lrn(y), 3, 2)
        else:
            y = self._conv0_col(x, relu=True) if col else self._conv(0, x, relu=True)
            for i in range(1, len(self.conv_specs)):
                y = self._conv(i, y, relu=True)
        B, TC, h, w = y.shape
        z = y.reshape(B, self.T, (TC // self.T) * h * w).transpose(0, 1)  # per-teacher NCHW flatten
        n = len(self.fc_w)
        for i in range(n):
            z = torch.baddbmm(self.fc_b[i].to(z.dtype), z, self.fc_w[i].to(z.dtype))
            if i + 1 < n:
                z = F.relu(z)
        return z

    # ------------------------------------------------------------------------ per-teacher I/O
    def teacher_state(self, t: int, tensors=None) -> dict:
        """Teacher t's PateCNN state_dict (from the parameters, or from `tensors` laid out like them)."""
        # parameters() order (registration order): conv weights, conv biases, fc weights, fc biases
        src = list(tensors) if tensors is not None else [p.detach() for p in self.parameters()]
        nconv = len(self.conv_specs)
        conv_w, conv_b = src[:nconv], src[nconv:2 * nconv]
        fc_w, fc_b = src[2 * nconv:2 * nconv + len(self.fc_names)], src[2 * nconv + len(self.fc_names):]
        out = {}
        for i, (name, _) in enumerate(self.conv_specs):
            co = conv_w[i].shape[0] // self.T
            out[f"{name}.weight"] = conv_w[i][t * co:(t + 1) * co]
            out[f"{name}.bias"] = conv_b[i][t * co:(t + 1) * co]
        for i, name in enumerate(self.fc_names):
            out[f"{name}.weight"] = fc_w[i][t].t()
            out[f"{name}.bias"] = fc_b[i][t, 0]
        return out

    def load_teachers(self, states: list[dict]) -> None:
        assert len(states) == self.T
        with torch.no_grad():
            for i, (name, _) in enumerate(self.conv_specs):
                self.conv_w[i].copy_(torch.cat([s[f"{name}.weight"] for s in states]))
                self.conv_b[i].copy_(torch.cat([s[f"{name}.bias"] for s in states]))
            for i, name in enumerate(self.fc_names):
                self.fc_w[i].copy_(torch.stack([s[f"{name}.weight"].t() for s in states]))
                self.fc_b[i].copy_(torch.stack([s[f"{name}.bias"].view(1, -1) for s in states]))


def _interleave(shards_x: list[np.ndarray], dev: torch.device) -> torch.Tensor:
    """T shards [n, H, W, C] (or [n, H, W]) -> one [n, T*C, H, W] batch tensor, channels_last storage."""
    xs = [np.asarray(s, np.float32) for s in shards_x]
    xs = [s[..., None] if s.ndim == 3 else s for s in xs]
    st = torch.as_tensor(np.stack(xs, 3))  # [n, H, W, T, C]
    n, h, w, T, c = st.shape
    t = st.reshape(n, h, w, T * c).to(dev).permute(0, 3, 1, 2)  # NCHW view of NHWC storage
    return t if dev.type == "cuda" else t.contiguous()


def _save_teacher(path: str, state: dict, ema: dict, step: int) -> None:
    import os

    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save({"step": step, "state_dict": {k: v.detach().cpu().clone() for k, v in state.items()},
                "ema": {k: v.detach().cpu().clone() for k, v in ema.items()}}, path)


def train_ensemble(shards_x: list[np.ndarray], shards_y: list[np.ndarray], ckpt_paths: list[str],
                   cfg: deep_cnn.DeepCNNConfig | None = None, device=None, log=print, checkpoint: bool = True,
                   step_times: list | None = None) -> bool:
    """Train len(shards_x) teachers together; teacher t's checkpoints go to `ckpt_paths[t]-<step>`, exactly as
    `deep_cnn.train(shards_x[t], shards_y[t], ckpt_paths[t], cfg)` writes them (`checkpoint=False`: none, for
    benchmarks; `step_times` collects the wall time of every step, device-synchronised)."""
    cfg = cfg or deep_cnn.DeepCNNConfig()
    T = len(shards_x)
    assert T == len(shards_y) == len(ckpt_paths) and T > 0
    n = len(shards_y[0])
    assert all(len(s) == n for s in shards_y) and all(len(s) == n for s in shards_x), "equal shard sizes"
    dev = deep_cnn._device(device)
    torch.manual_seed(cfg.dropout_seed)  # the sequential trainer's per-teacher initialisation
    template = deep_cnn.build_model(cfg)
    ens = PateEnsemble(template, T).to(dev)
    x = _interleave(shards_x, dev).to(ens.conv_w[0].dtype)
    col = ens.col_input
    if col:  # im2col image of the resident dataset, built once
        x = ens.conv_input(x)
    y = torch.as_tensor(np.stack([np.asarray(s) for s in shards_y])).to(dev).long()  # [T, n]
    params = list(ens.parameters())
    nb_ex_per_epoch = int(60000 / cfg.nb_teachers)
    decay_steps = max(1, int(nb_ex_per_epoch / cfg.batch_size * cfg.epochs_per_decay))
    lr0 = float(cfg.learning_rate) / 100.0
    opt = cnn_ops.SGDEMA(params, lr=lr0, ema=True)
    nb_batches = math.ceil(n / cfg.batch_size)
    amp = dev.type == "cuda"
    for step in range(cfg.max_steps):
        t0 = time.time()
        lr = lr0 * deep_cnn.LEARNING_RATE_DECAY_FACTOR ** (step // decay_steps)
        s, e = deep_cnn.batch_indices(step % nb_batches, n, cfg.batch_size)
        opt.zero_grad()
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=amp):
            logits = ens(x[s:e], col=col)  # [T, B, classes]
        B = e - s
        # sum over teachers of each teacher's mean loss: teacher t's gradient is its own mean-loss gradient
        loss = cnn_ops.softmax_cross_entropy(logits.float().reshape(T * B, -1), y[:, s:e].reshape(-1),
                                             reduction="sum") / B
        loss.backward()
        decay = min(deep_cnn.MOVING_AVERAGE_DECAY, (1.0 + step) / (10.0 + step))
        opt.step(lr=lr, decay=decay)
        if step_times is not None:
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            step_times.append(time.time() - t0)
        if step % cfg.log_every == 0 or step % cfg.ckpt_every == 0 or step + 1 == cfg.max_steps:
            loss_value = float(loss.detach()) / T
            assert not np.isnan(loss_value), "Model diverged with loss = NaN"
            if step % cfg.log_every == 0:
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                dur = time.time() - t0
                log(f"{datetime.now()}: step {step}, mean teacher loss = {loss_value:.2f} "
                    f"({T * cfg.batch_size / max(dur, 1e-9):.1f} examples/sec over {T} teachers; {dur:.3f} sec/batch)")
            if checkpoint and (step % cfg.ckpt_every == 0 or step + 1 == cfg.max_steps):
                for t in range(T):
                    _save_teacher(f"{ckpt_paths[t]}-{step}", ens.teacher_state(t), ens.teacher_state(t, opt.shadow),
                                  step)
    return True


@torch.no_grad()
def ensemble_softmax_preds(images: np.ndarray, ckpt_paths: list[str], cfg: deep_cnn.DeepCNNConfig | None = None,
                           device=None, batch: int = 1024) -> np.ndarray:
    """[T, N, classes] softmax predictions of every teacher's EMA weights on the same images, one grouped forward
    per batch (the per-teacher loop of `train_student.ensemble_preds`, `deep_cnn.softmax_preds` semantics)."""
    cfg = cfg or deep_cnn.DeepCNNConfig()
    dev = deep_cnn._device(device)
    states = []
    for p in ckpt_paths:
        ck = torch.load(p, map_location="cpu", weights_only=True)
        st = dict(ck["state_dict"])
        st.update(ck["ema"])
        states.append(st)
    T = len(states)
    ens = PateEnsemble(deep_cnn.build_model(cfg), T)
    ens.load_teachers(states)
    ens = ens.to(dev).eval()
    imgs = torch.as_tensor(np.asarray(images, np.float32))
    if imgs.dim() == 3:
        imgs = imgs.unsqueeze(-1)  # [N, H, W, C]
    outs = []
    for i in range(0, len(imgs), batch):
        xb = imgs[i:i + batch].to(dev, ens.conv_w[0].dtype)
        nb, h, w, c = xb.shape  # every teacher sees the same images: replicate along the teacher channel blocks
        xb = xb.unsqueeze(3).expand(nb, h, w, T, c).reshape(nb, h, w, T * c).permute(0, 3, 1, 2)
        if dev.type != "cuda":
            xb = xb.contiguous()
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
            o = (ens(ens.conv_input(xb), col=True) if ens.col_input else ens(xb)).float()
        outs.append(F.softmax(o, -1))
    return torch.cat(outs, 1).cpu().numpy().astype(np.float32)
