"""Small-CNN kernels (csrc/cnn_ops.hip) vs fp32 PyTorch references: fused softmax cross-entropy,
TF-semantics LRN forward/backward, fused SGD + EMA."""
import math

import pytest
import torch
import torch.nn.functional as F

from mifx.ops import cnn_ops


def _tf_lrn_ref(x, r, bias, alpha, beta):
    """Direct tf.nn.lrn formula over dim 1 (fp64 loop-free reference)."""
    sq = x.pow(2)
    C = x.shape[1]
    s = torch.zeros_like(x)
    for c in range(C):
        lo, hi = max(0, c - r), min(C - 1, c + r)
        s[:, c] = sq[:, lo:hi + 1].sum(1)
    return x / (bias + alpha * s).pow(beta)


def test_cpu_lrn_matches_tf_formula():
    x = torch.randn(2, 13, 5, 4, dtype=torch.float64)
    got = cnn_ops.lrn(x, 4, 1.0, 0.001 / 9.0, 0.75)
    torch.testing.assert_close(got, _tf_lrn_ref(x, 4, 1.0, 0.001 / 9.0, 0.75))
    x = torch.randn(2, 7, 3, 3, dtype=torch.float64) * 5
    torch.testing.assert_close(cnn_ops.lrn(x, 2, 2.0, 0.3, 0.5), _tf_lrn_ref(x, 2, 2.0, 0.3, 0.5))


def test_cpu_softmax_xent_reference():
    x, y = torch.randn(6, 10), torch.tensor([1, 2, 3, -100, 0, 9])
    torch.testing.assert_close(cnn_ops.softmax_cross_entropy(x, y), F.cross_entropy(x, y))
    torch.testing.assert_close(cnn_ops.softmax_cross_entropy(x, y, "none"), F.cross_entropy(x, y, reduction="none"))


def test_cpu_sgd_ema_matches_formula():
    p = torch.nn.Parameter(torch.randn(100))
    p.grad = torch.randn(100)
    w0, g0 = p.detach().clone(), p.grad.clone()
    opt = cnn_ops.SGDEMA([p], lr=0.1, weight_decay=0.01)
    opt.step(decay=0.9)
    w1 = w0 - 0.1 * (g0 + 0.01 * w0)
    torch.testing.assert_close(p.detach(), w1)
    torch.testing.assert_close(opt.shadow[0], w0 + 0.1 * (w1 - w0))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,C", [(torch.float32, 10), (torch.bfloat16, 10), (torch.float32, 1001),
                                     (torch.float32, 3)])
@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_gpu_softmax_xent_matches_torch(dtype, C, reduction):
    torch.manual_seed(C)
    B = 777
    x = (torch.randn(B, C, device="cuda") * 3).to(dtype)
    y = torch.randint(0, C, (B,), device="cuda")
    y[::50] = -100  # ignore_index rows
    xa = x.clone().requires_grad_()
    xr = x.float().clone().requires_grad_()
    la = cnn_ops.softmax_cross_entropy(xa, y, reduction)
    lr = F.cross_entropy(xr, y, reduction=reduction)
    tol = 1e-5 if dtype == torch.float32 else 2e-2
    torch.testing.assert_close(la.float(), lr, rtol=tol, atol=tol)
    g = torch.randn_like(lr)
    la.backward(g)
    lr.backward(g)
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=tol, atol=tol * (1.0 / B if reduction == "mean" else 1))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("C", [64, 128, 37])
@pytest.mark.parametrize("alpha", [0.001 / 9.0, 0.05])
def test_gpu_lrn_matches_reference(dtype, tol, C, alpha):
    """bf16 C=64/128 take the vectorised kernels (normaliser recomputed in backward), the rest the generic ones."""
    torch.manual_seed(C)
    r, bias, beta = 4, 1.0, 0.75
    x = (torch.randn(8, C, 14, 14, device="cuda") * 4).to(dtype).contiguous(memory_format=torch.channels_last)
    xa = x.clone().requires_grad_()
    x64 = x.double().clone().requires_grad_()
    ya = cnn_ops.lrn(xa, r, bias, alpha, beta)
    assert ya.is_contiguous(memory_format=torch.channels_last)
    y64 = _tf_lrn_ref(x64, r, bias, alpha, beta)
    torch.testing.assert_close(ya.double(), y64, rtol=tol, atol=tol)
    g = torch.randn_like(y64).to(dtype)
    ya.backward(g)
    y64.backward(g.double())
    torch.testing.assert_close(xa.grad.double(), x64.grad, rtol=tol * 3, atol=tol * 3)


@pytest.mark.gpu
def test_gpu_sgd_ema_matches_formula():
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(n, device="cuda")) for n in (5, 8192, 8193, 100000)]
    for p in ps:
        p.grad = torch.randn_like(p)
    w0 = [p.detach().clone() for p in ps]
    opt = cnn_ops.SGDEMA(ps, lr=0.05, weight_decay=1e-3)
    assert opt.native
    for step in range(3):
        decay = min(0.9999, (1.0 + step) / (10.0 + step))
        ref_w = [w - 0.05 * (p.grad + 1e-3 * w) for w, p in zip(w0, ps)]
        ref_s = [s + (1 - decay) * (w - s) for s, w in zip([s.clone() for s in opt.shadow], ref_w)]
        opt.step(decay=decay)
        for p, rw in zip(ps, ref_w):
            torch.testing.assert_close(p.detach(), rw, rtol=1e-6, atol=1e-6)
        for s, rs in zip(opt.shadow, ref_s):
            torch.testing.assert_close(s, rs, rtol=1e-6, atol=1e-6)
        w0 = [p.detach().clone() for p in ps]


@pytest.mark.gpu
def test_gpu_pate_cnn_train_step_uses_native_ops():
    """PATE deep_cnn training on the GPU: LRN + softmax-CE + SGD/EMA kernels, finite decreasing loss."""
    import numpy as np

    from mifx.privacy.pate import deep_cnn

    x = np.random.default_rng(0).random((512, 28, 28, 1), dtype=np.float32)
    y = (x.reshape(512, -1).mean(1) * 1000).astype(np.int64) % 10
    cfg = deep_cnn.DeepCNNConfig(max_steps=30, batch_size=128, log_every=10, ckpt_every=1000, nb_teachers=50)
    lines = []
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        assert deep_cnn.train(x, y, f"{d}/m.ckpt", cfg, device="cuda", log=lines.append)
        preds = deep_cnn.softmax_preds(x[:64], f"{d}/m.ckpt-29", cfg, device="cuda")
    assert preds.shape == (64, 10) and np.allclose(preds.sum(1), 1, atol=1e-3)
    losses = [float(ln.split("loss = ")[1].split(" ")[0]) for ln in lines]
    assert all(math.isfinite(v) for v in losses)
