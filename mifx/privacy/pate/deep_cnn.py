"""PATE-2017 teacher/student CNN training and inference (reference
`research/pate_2017/deep_cnn.py:375-603`, `input.py:90-118,397-424`, `utils.py:17-35`).

Behaviour kept from the reference:
  * SGD with staircase exponential decay: lr0 = learning_rate/100, x0.1 every
    `epochs_per_decay` epochs of a 60000/nb_teachers-example shard (`train_op_fun`).
  * Exponential moving average of every trainable weight with TF's num_updates rule
    (decay = min(0.9999, (1+step)/(10+step))); inference restores the EMA shadow weights.
  * Sequential batches with the reference's wrap-around `batch_indices`, NaN-loss assert,
    an examples/sec + sec/batch line every 100 steps, a checkpoint every 1000 steps and at
    the last step (`<ckpt_path>-<step>`).

MI355X-first choices: the model runs NHWC (channels_last) under bf16 autocast on the GPU
(MIOpen MFMA implicit-GEMM convolutions), the whole shard is resident in HBM, and the EMA
update is fused with the SGD step into one multi-tensor HIP kernel (`cnn_ops.SGDEMA`); the softmax
cross-entropy head and the LRN layers run as HIP kernels too (csrc/cnn_ops.hip)."""
from __future__ import annotations

import math
import os
import time
from dataclasses import dataclass
from datetime import datetime

import numpy as np
import torch
import torch.nn.functional as F

from ...models.cnn import PateCNN
from ...ops import cnn_ops

MOVING_AVERAGE_DECAY = 0.9999
LEARNING_RATE_DECAY_FACTOR = 0.1


@dataclass
class DeepCNNConfig:
    dataset: str = "mnist"
    nb_labels: int = 10
    batch_size: int = 128
    epochs_per_decay: int = 350
    learning_rate: int = 5  # x100, as the reference flag
    max_steps: int = 3000
    nb_teachers: int = 50
    deeper: bool = False
    dropout_seed: int = 123
    log_every: int = 100
    ckpt_every: int = 1000


def batch_indices(batch_nb: int, data_length: int, batch_size: int) -> tuple[int, int]:
    """Start/end of batch `batch_nb`; the last batch is shifted back to stay full."""
    start, end = int(batch_nb * batch_size), int((batch_nb + 1) * batch_size)
    if end > data_length:
        shift = end - data_length
        start, end = start - shift, end - shift
    return start, end


def image_whitening(data: np.ndarray) -> np.ndarray:
    """Per-image mean subtraction and division by max(std, 1/sqrt(#pixels)) on [N, H, W, C]."""
    assert data.ndim == 4
    data = data.astype(np.float32, copy=True)
    nb_pixels = data.shape[1] * data.shape[2] * data.shape[3]
    data -= data.mean(axis=(1, 2, 3), keepdims=True)
    adj = np.maximum(np.float32(1.0 / math.sqrt(nb_pixels)), data.std(axis=(1, 2, 3), keepdims=True))
    return data / adj


def partition_dataset(data, labels, nb_teachers: int, teacher_id: int):
    assert len(data) == len(labels) and int(teacher_id) < int(nb_teachers)
    n = int(len(data) / nb_teachers)
    return data[teacher_id * n:(teacher_id + 1) * n], labels[teacher_id * n:(teacher_id + 1) * n]


def load_dataset(dataset: str, seed: int = 0, train_size: int | None = None, test_size: int | None = None):
    """Synthetic stand-ins with the reference datasets' shapes (no downloads offline):
    mnist 28x28x1 (60000/10000), svhn/cifar10 32x32x3. Returns NHWC float32 + int32 labels."""
    shapes = {"mnist": ((28, 28), 1, 60000, 10000), "svhn": ((32, 32), 3, 73257, 26032),
              "cifar10": ((32, 32), 3, 50000, 10000)}
    if dataset not in shapes:
        raise ValueError(f"unknown dataset {dataset!r}")
    from ...data.synthetic import synthetic_images

    hw, ch, ntr, nte = shapes[dataset]
    ntr, nte = train_size or ntr, test_size or nte
    x, y = synthetic_images(ntr + nte, shape=hw, channels=ch, seed=seed)
    x = x.reshape(len(x), ch, *hw).permute(0, 2, 3, 1).contiguous().numpy()
    if dataset != "mnist":
        x = image_whitening(x)
    y = y.numpy().astype(np.int32)
    return x[:ntr], y[:ntr], x[ntr:], y[ntr:]


def build_model(cfg: DeepCNNConfig, dropout: bool = False) -> PateCNN:
    ch, img = (1, 28) if cfg.dataset == "mnist" else (3, 32)
    return PateCNN(in_ch=ch, num_classes=cfg.nb_labels, image=img, deeper=cfg.deeper, dropout=dropout)


def _device(device) -> torch.device:
    return torch.device(device or ("cuda" if torch.cuda.is_available() else "cpu"))


def _to_nchw(x: np.ndarray, dev: torch.device) -> torch.Tensor:
    t = torch.as_tensor(x, device=dev)
    if t.dim() == 3:
        t = t.unsqueeze(-1)
    t = t.permute(0, 3, 1, 2)  # NHWC storage viewed as NCHW == channels_last
    return t.contiguous(memory_format=torch.channels_last) if dev.type == "cuda" else t.contiguous()


def _save(path: str, model, shadow, step: int) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    names = [n for n, _ in model.named_parameters()]
    torch.save({"step": step, "state_dict": {k: v.detach().cpu() for k, v in model.state_dict().items()},
                "ema": {n: s.detach().cpu() for n, s in zip(names, shadow)}}, path)


def train(images: np.ndarray, labels: np.ndarray, ckpt_path: str, cfg: DeepCNNConfig | None = None,
          dropout: bool = False, device=None, log=print) -> bool:
    cfg = cfg or DeepCNNConfig()
    assert len(images) == len(labels)
    dev = _device(device)
    torch.manual_seed(cfg.dropout_seed)
    model = build_model(cfg, dropout).to(dev)
    if dev.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    pdt = next(model.parameters()).dtype  # fp32 (fp64 in the ensemble-equivalence test)
    x = _to_nchw(np.asarray(images, np.float32), dev).to(pdt)
    y = torch.as_tensor(np.asarray(labels), device=dev).long()
    params = [p for p in model.parameters() if p.requires_grad]
    nb_ex_per_epoch = int(60000 / cfg.nb_teachers)
    decay_steps = max(1, int(nb_ex_per_epoch / cfg.batch_size * cfg.epochs_per_decay))
    lr0 = float(cfg.learning_rate) / 100.0
    # SGD + EMA shadow update in one multi-tensor HIP launch on the GPU (csrc/cnn_ops.hip)
    opt = cnn_ops.SGDEMA(params, lr=lr0, ema=True)
    shadow = opt.shadow
    n = len(x)
    nb_batches = math.ceil(n / cfg.batch_size)
    amp = dev.type == "cuda"
    model.train()
    for step in range(cfg.max_steps):
        t0 = time.time()
        lr = lr0 * LEARNING_RATE_DECAY_FACTOR ** (step // decay_steps)  # staircase exponential decay
        s, e = batch_indices(step % nb_batches, n, cfg.batch_size)
        opt.zero_grad()
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=amp):
            logits = model(x[s:e])
        loss = cnn_ops.softmax_cross_entropy(logits.float(), y[s:e])  # fused loss + dlogits
        loss.backward()
        decay = min(MOVING_AVERAGE_DECAY, (1.0 + step) / (10.0 + step))
        opt.step(lr=lr, decay=decay)
        if step % cfg.log_every == 0 or step % cfg.ckpt_every == 0 or step + 1 == cfg.max_steps:
            loss_value = float(loss.detach())  # host sync only on logging / checkpoint steps
            assert not np.isnan(loss_value), "Model diverged with loss = NaN"
            if step % cfg.log_every == 0:
                if dev.type == "cuda":
                    torch.cuda.synchronize()
                dur = time.time() - t0
                log(f"{datetime.now()}: step {step}, loss = {loss_value:.2f} "
                    f"({cfg.batch_size / max(dur, 1e-9):.1f} examples/sec; {dur:.3f} sec/batch)")
            if step % cfg.ckpt_every == 0 or step + 1 == cfg.max_steps:
                _save(f"{ckpt_path}-{step}", model, shadow, step)
    return True


@torch.no_grad()
def softmax_preds(images: np.ndarray, ckpt_path: str, cfg: DeepCNNConfig | None = None, return_logits: bool = False,
                  device=None) -> np.ndarray:
    """Predictions of the EMA shadow weights stored at `ckpt_path` (batched by cfg.batch_size)."""
    cfg = cfg or DeepCNNConfig()
    dev = _device(device)
    ck = torch.load(ckpt_path, map_location="cpu", weights_only=True)
    model = build_model(cfg).to(dev)
    model.load_state_dict(ck["state_dict"])
    for name, p in model.named_parameters():
        p.copy_(ck["ema"][name])
    if dev.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    model.eval()
    x = _to_nchw(np.asarray(images, np.float32), dev).to(next(model.parameters()).dtype)
    outs = []
    bs = max(cfg.batch_size, 4096)
    for i in range(0, len(x), bs):
        with torch.autocast(dev.type, dtype=torch.bfloat16, enabled=dev.type == "cuda"):
            o = model(x[i:i + bs]).float()
        outs.append(o if return_logits else F.softmax(o, -1))
    return torch.cat(outs).cpu().numpy().astype(np.float32)
