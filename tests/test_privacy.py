"""Differential privacy: accountant goldens + mpmath oracle, queries, DP optimizers, PATE analyses.

Reference strategy: `analysis/rdp_accountant_test.py` (goldens + mpmath quadrature of
A_alpha), `optimizers/dp_optimizer_test.py` (exact grads for M=1,2,4 without noise, clipping to
[-0.6,-0.8], noise std ~ C*sigma over 1000 draws), `gaussian_query_test.py`,
`nested_query_test.py`, `pate_2018/core_test.py`, `pate_2018/smooth_sensitivity_test.py`
(numeric goldens). GPU tests compare the HIP kernels with the bit-compatible host Philox path."""
import math
import sys

import mpmath as mp
import numpy as np
import pytest
import torch

from mifx.ops import dp as dpops
from mifx.privacy import queries as Q
from mifx.privacy import rdp
from mifx.privacy.optimizers import DPAdagradOptimizer, DPAdamOptimizer, DPGradientDescentOptimizer
from mifx.privacy.pate import aggregation, analysis2017, rdp2018
from mifx.privacy.pate import smooth_sensitivity as ss

# ---------------------------------------------------------------- accountant


def test_rdp_trivial_cases():
    assert rdp.compute_rdp(0, 10, 1, 20) == 0
    assert rdp.compute_rdp(1, 10, 1, 20) == 0.1


def test_rdp_scalar_and_sequence_goldens():
    assert rdp.compute_rdp(0.1, 2, 10, 5) == pytest.approx(0.07737, abs=5e-6)
    got = rdp.compute_rdp(0.01, 2.5, 50, [1.5, 2.5, 5, 50, 100, np.inf])
    np.testing.assert_allclose(got[:5], [0.00065, 0.001085, 0.00218075, 0.023846, 167.416307], atol=1e-5)
    assert np.isinf(got[5])


def _a_mp(sigma, q, alpha):
    mu0 = lambda x: mp.npdf(x, mu=0, sigma=sigma)  # noqa: E731
    ratio = lambda x: (1 - q) + q * mp.exp((2 * x - 1) / (2 * sigma ** 2))  # noqa: E731
    return mp.quad(lambda z: mu0(z) * ratio(z) ** alpha, (-mp.inf, mp.inf), maxdegree=8)


@pytest.mark.parametrize("q,sigma,order", [(1e-7, .1, 1.01), (1e-6, .1, 256), (1e-5, .1, 256.1), (1e-6, 1, 27),
                                           (1e-4, 1., 1.5), (1e-3, 1., 2), (.01, 10, 20), (.1, 100, 20.5),
                                           (.99, .1, 256), (.999, 100, 256.1)])
def test_log_a_matches_mpmath(q, sigma, order):
    a = _a_mp(sigma, q, order)
    ref = float(mp.log(a)) if a >= sys.float_info.min else -np.inf
    np.testing.assert_allclose(rdp.log_a(q, sigma, order), ref, rtol=1e-4)


def test_privacy_spent_goldens():
    orders = range(2, 33)
    r = rdp.compute_rdp(0.01, 4, 10000, orders)
    eps, _, order = rdp.get_privacy_spent(orders, r, target_delta=1e-5)
    assert eps == pytest.approx(1.258575, abs=5e-6) and order == 20
    _, delta, order = rdp.get_privacy_spent(orders, r, target_eps=1.258575)
    assert delta == pytest.approx(1e-5, abs=1e-7) and order == 20


def test_composition_golden():
    orders = (1.25, 1.5, 1.75, 2., 2.5, 3., 4., 5., 6., 7., 8., 10., 12., 14., 16., 20., 24., 28., 32., 64., 256.)
    r = rdp.compute_rdp(q=1e-4, noise_multiplier=.4, steps=40000, orders=orders)
    r = r + rdp.compute_rdp(q=0.1, noise_multiplier=2, steps=100, orders=orders)
    eps, _, order = rdp.get_privacy_spent(orders, r, target_delta=1e-5)
    assert eps == pytest.approx(8.509656, abs=5e-6) and order == 2.5
    acc = rdp.RdpAccountant(orders)
    acc.step(1e-4, .4, 40000)
    acc.step(0.1, 2, 100)
    assert acc.epsilon(1e-5) == pytest.approx(8.509656, abs=5e-6)


NOTEBOOK_ORDERS = [1.25, 1.5, 1.75, 2., 2.25, 2.5, 3., 3.5, 4., 4.5] + list(range(5, 64)) + [128, 256, 512]


def _notebook_analysis(n, batch, sigma, epochs, delta=1e-5):
    """apply_dp_sgd_analysis of notebooks/privacy/TensorFlow_Privacy.ipynb (cell 3), same order list."""
    import math

    q = batch / n
    steps = int(math.ceil(epochs * n / batch))
    eps, _, order = rdp.get_privacy_spent(NOTEBOOK_ORDERS, rdp.compute_rdp(q, sigma, steps, NOTEBOOK_ORDERS),
                                          target_delta=delta)
    return eps, order


def test_notebook_privacy_statement_2_92():
    """The notebook's markdown (TensorFlow_Privacy.ipynb cell 2) states "(2.92, 1e-5)-DP". That figure is the
    TF-Privacy MNIST tutorial configuration (N=60000, B=256, sigma=1.12, 60 epochs) run through the notebook's
    own analysis cell; we reproduce it to 3 digits. The cell's printed output for its local variables
    (N=600, B=32, sigma=1.12, 1 epoch) is not recorded in the reference: ours is eps=2.487 at order 7
    (parity unpinned, pinned here as a regression value)."""
    eps, _ = _notebook_analysis(60000, 256, 1.12, 60)
    assert round(eps, 2) == 2.92
    eps_nb, order_nb = _notebook_analysis(600, 32, 1.12, 1)
    assert eps_nb == pytest.approx(2.48666, abs=1e-4) and order_nb == 7


def test_dp_sgd_tutorial_epsilon_is_sane():
    eps, _ = rdp.compute_dp_sgd_privacy(60000, 256, 1.1, 60, 1e-5)
    assert 2.0 < eps < 4.0  # the tutorial reports eps ~= 3 for these settings


# ---------------------------------------------------------------- queries


def _run_query(query, records):
    gs = query.initial_global_state()
    params = query.derive_sample_params(gs)
    st = query.initial_sample_state(gs, records[0])
    for r in records:
        st = query.accumulate_record(params, st, r)
    return query.get_query_result(st, gs)


def test_gaussian_sum_no_clip_no_noise():
    r = [torch.tensor([1.0, 1.0]), torch.tensor([3.0, 4.0])]
    res, _ = _run_query(Q.GaussianSumQuery(10.0, 0.0), r)
    torch.testing.assert_close(res, torch.tensor([4.0, 5.0]))


def test_gaussian_sum_with_clip():
    r = [torch.tensor([-6.0, 8.0]), torch.tensor([4.0, -3.0])]  # norms 10 and 5
    res, _ = _run_query(Q.GaussianSumQuery(5.0, 0.0), r)
    torch.testing.assert_close(res, torch.tensor([1.0, 1.0]))


def test_gaussian_sum_noise_std():
    g = torch.Generator().manual_seed(1)
    q = Q.GaussianSumQuery(5.0, 1.0, generator=g)
    vals = [float(_run_query(q, [torch.tensor([0.0])])[0]) for _ in range(1000)]
    assert np.std(vals) == pytest.approx(1.0, abs=0.1)


def test_gaussian_average_and_nested():
    r = [torch.tensor([1.0, 1.0]), torch.tensor([3.0, 4.0])]
    res, _ = _run_query(Q.GaussianAverageQuery(10.0, 0.0, 2.0), r)
    torch.testing.assert_close(res, torch.tensor([2.0, 2.5]))
    nested = Q.NestedQuery([Q.GaussianSumQuery(10.0, 0.0), {"a": Q.NoPrivacySumQuery()}])
    recs = [[torch.tensor([1.0]), {"a": (torch.tensor([2.0]), torch.tensor([3.0]))}],
            [torch.tensor([4.0]), {"a": (torch.tensor([5.0]), torch.tensor([6.0]))}]]
    out, _ = _run_query(nested, recs)
    torch.testing.assert_close(out[0], torch.tensor([5.0]))
    torch.testing.assert_close(out[1]["a"][1], torch.tensor([9.0]))
    with pytest.raises(ValueError):
        _run_query(nested, [[torch.tensor([1.0])]])


def test_no_privacy_average_weighted():
    q = Q.NoPrivacyAverageQuery()
    gs = q.initial_global_state()
    st = q.initial_sample_state(gs, torch.zeros(1))
    st = q.accumulate_record(None, st, torch.tensor([2.0]), weight=1.0)
    st = q.accumulate_record(None, st, torch.tensor([5.0]), weight=3.0)
    torch.testing.assert_close(q.get_query_result(st, gs)[0], torch.tensor([17.0 / 4.0]))


# ---------------------------------------------------------------- DP optimizers


class _Var(torch.nn.Module):
    """out = v - data, so loss 0.5*||out||^2 is the reference's 0.5*sum((v - data)^2) per example."""

    def __init__(self, init):
        super().__init__()
        self.v = torch.nn.Parameter(torch.tensor(init))

    def forward(self, data):
        return self.v - data


def _half_sq(out, _t):
    return 0.5 * (out ** 2).sum(-1)


@pytest.mark.parametrize("cls", [DPGradientDescentOptimizer, DPAdagradOptimizer, DPAdamOptimizer])
@pytest.mark.parametrize("m,expected", [(1, [-10.0, -10.0]), (2, [-5.0, -5.0]), (4, [-2.5, -2.5])])
def test_dp_optimizer_baseline(cls, m, expected):
    model = _Var([1.0, 2.0])
    data = torch.tensor([[3.0, 4.0], [5.0, 6.0], [7.0, 8.0], [-1.0, 0.0]])
    opt = cls(l2_norm_clip=1.0e9, noise_multiplier=0.0, num_microbatches=m, params=model.parameters(),
              learning_rate=2.0)
    opt.compute_gradients(model, _half_sq, data, torch.zeros(4))
    torch.testing.assert_close(model.v.grad, torch.tensor(expected))


@pytest.mark.parametrize("cls", [DPGradientDescentOptimizer, DPAdagradOptimizer, DPAdamOptimizer])
def test_dp_optimizer_clipping(cls):
    model = _Var([0.0, 0.0])
    data = torch.tensor([[3.0, 4.0], [6.0, 8.0]])
    opt = cls(l2_norm_clip=1.0, noise_multiplier=0.0, num_microbatches=1, params=model.parameters(),
              learning_rate=2.0)
    opt.compute_gradients(model, _half_sq, data, torch.zeros(2))
    torch.testing.assert_close(model.v.grad, torch.tensor([-0.6, -0.8]))


def test_dp_optimizer_noise_std():
    model = _Var([0.0])
    data = torch.tensor([[0.0]])
    opt = DPGradientDescentOptimizer(l2_norm_clip=4.0, noise_multiplier=2.0, num_microbatches=1,
                                     params=model.parameters(), learning_rate=2.0, seed=3)
    grads = []
    for i in range(1000):
        opt.steps = i  # a fresh Philox offset per draw
        opt.compute_gradients(model, _half_sq, data, torch.zeros(1))
        grads.append(float(model.v.grad))
    assert np.std(grads) == pytest.approx(8.0, abs=0.5)


def test_dp_optimizer_chunked_equals_fused():
    torch.manual_seed(0)
    from mifx.models.cnn import MnistDPCNN

    def run(max_bytes):
        torch.manual_seed(0)
        m = MnistDPCNN()
        opt = DPGradientDescentOptimizer(1.0, 1.1, 8, m.parameters(), 0.1, seed=11)
        opt.max_g_bytes = max_bytes
        x = torch.randn(16, 28, 28, generator=torch.Generator().manual_seed(2))
        y = torch.randint(0, 10, (16,), generator=torch.Generator().manual_seed(3))
        loss = opt.step(m, lambda out, t: torch.nn.functional.cross_entropy(out, t, reduction="none"), x, y)
        return float(loss), [p.detach().clone() for p in m.parameters()]

    l1, p1 = run(8 << 30)
    l2, p2 = run(26010 * 4 * 3)  # 3 microbatches per chunk
    assert l1 == pytest.approx(l2, rel=1e-6)
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


# ---------------------------------------------------------------- noise streams


def test_philox_known_answer():
    # Philox4x32-10 known-answer vector (Random123): counter 0, key 0
    x = dpops.philox4x32(0, 0, 0, 0, 0)
    assert [int(v) for v in x] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_clip_sum_noise_cpu_semantics():
    G = torch.tensor([[3.0, 4.0], [0.3, 0.4]])
    out = dpops.clip_sum_noise(G, 1.0, 0.0, 2.0)
    torch.testing.assert_close(out, torch.tensor([(0.6 + 0.3) / 2, (0.8 + 0.4) / 2]))


# ---------------------------------------------------------------- PATE


def test_noisy_max_cpu_and_clean_votes():
    T, N, C = 50, 40, 10
    r = np.random.default_rng(0)
    truth = r.integers(0, C, N)
    labels = np.where(r.random((T, N)) < 0.8, truth[None, :], r.integers(0, C, (T, N))).astype(np.int32)
    out, votes, lab = aggregation.noisy_max(labels, 1.0, return_clean_votes=True)
    assert votes.sum(axis=1).tolist() == [T] * N and np.array_equal(lab, labels)
    assert aggregation.accuracy(out, truth) > 0.95
    probs = np.eye(C)[labels]  # [T, N, C] one-hot teacher outputs
    assert np.array_equal(aggregation.aggregation_most_frequent(probs), np.argmax(votes, axis=1))


def test_pate2017_analysis_behaviour():
    strong = np.array([240, 5, 5] + [0] * 7)
    weak = np.array([90, 80, 80] + [0] * 7)
    assert analysis2017.compute_q_noisy_max(strong, 0.1) < analysis2017.compute_q_noisy_max(weak, 0.1)
    rep = analysis2017.analyze(np.stack([strong] * 100), noise_eps=0.1, delta=1e-5)
    assert rep["eps"] < rep["data_independent_eps"]


def test_pate2018_core_value_errors_and_monotonicity():
    with pytest.raises(ValueError):
        rdp2018.rdp_gaussian(1.0, 1.0, np.array([2, 3, 4]))
    with pytest.raises(ValueError):
        rdp2018.rdp_gaussian(np.log(0.5), -1.0, np.array([2, 3, 4]))
    with pytest.raises(ValueError):
        rdp2018.rdp_gaussian(np.log(0.5), 1.0, np.array([1, 3, 4]))
    with pytest.raises(ValueError):
        rdp2018.compute_eps_from_delta([1.1, 2, 3, 4], [1, 2, 3], 0.001)
    neglogq0s = [2.8, 2.6, 427, None, 4.8, 4.0, 4.7, 275, 9.6, 8.8, 6.0, 4, 12, 11.2, 8.6, 6.4]
    k = 0
    for sigma in [1.5, 15, 1500, 15000]:
        for order in [1.1, 2.5, 32, 250]:
            nq = neglogq0s[k]
            k += 1
            if nq is None:
                continue
            at_q0 = rdp2018.rdp_gaussian(-nq, sigma, order)
            lq = -nq - np.array([0, np.log(2), np.log(4), np.log(8)])
            for i in range(3):
                assert rdp2018.rdp_gaussian(lq[i], sigma, order) > rdp2018.rdp_gaussian(lq[i + 1], sigma, order)
            for q in np.exp(-nq) + np.array([0.1, 0.2, 0.3, 0.4]):
                assert rdp2018.rdp_gaussian(np.log(q), sigma, order) == at_q0
    for sigma in [1e-3, 1.0, 1e5]:
        orders = [1.1, 2.5, 250.0]
        eps = [rdp2018.compute_eps_from_delta(orders, np.array(orders) / (2 * sigma ** 2), d)[0]
               for d in [1e-60, 1e-6, 0.1, 0.999]]
        assert eps == sorted(eps, reverse=True)


def test_smooth_sensitivity_gnmax_goldens():
    out1 = ss.compute_local_sensitivity_bounds_gnmax(np.array([10, 0, 0]), 10, .5, 1.5)
    np.testing.assert_allclose(out1, [3.13503646e-17, 1.60178280e-08, 5.90681786e-03] + [5.99981308e+00] * 7,
                               rtol=1e-8, atol=0)
    out2 = ss.compute_local_sensitivity_bounds_gnmax(np.array([1000, 500, 300, 200, 0]), 2000, 250., 10.)
    np.testing.assert_allclose(out2, [0.] * 298 + [2.77693450548e-7, 2.10853979548e-6] + [2.73113623988e-6] * 1700,
                               rtol=1e-8, atol=0)


def test_smooth_sensitivity_threshold_goldens():
    c = np.array([20, 10, 0])
    n = int(c.sum())
    out1 = ss.compute_local_sensitivity_bounds_threshold(c, n, 16, 2, 10)
    ans1 = [0] * 3 + [1.48454129e-04, 1.47826870e-02, 3.94153241e-02, 6.45775697e-02, 9.01543247e-02,
                      1.16054002e-01, 1.42180452e-01, 1.42180452e-01, 1.48454129e-04, 1.47826870e-02,
                      3.94153241e-02, 6.45775697e-02, 9.01543266e-02, 1.16054000e-01, 1.42180452e-01,
                      1.68302106e-01, 1.93127860e-01] + [0] * 10
    # two golden entries carry scipy-version noise in the 8th digit (9.01543247e-02 vs ...266e-02)
    np.testing.assert_allclose(out1, ans1, rtol=5e-8, atol=0)
    out3 = ss.compute_local_sensitivity_bounds_threshold(c, n, 50, 2, 10)
    ans3 = [1.35750725752e-19, 1.88990500499e-17, 2.05403154065e-15, 1.74298153642e-13, 1.15489723995e-11,
            5.97584949325e-10, 2.41486826748e-08, 7.62150641922e-07, 1.87846248741e-05, 0.000360973025976,
            0.000360973025976, 2.76377015215e-50, 1.00904975276e-53, 2.87254164748e-57, 6.37583360761e-61,
            1.10331620211e-64, 1.48844393335e-68, 1.56535552444e-72, 1.28328011060e-76, 8.20047697109e-81] + [0] * 10
    np.testing.assert_allclose(out3, ans3, rtol=1e-8, atol=0)
    out4 = ss.compute_local_sensitivity_bounds_threshold(np.array([19.5, -5.1, 0]), n, 10.1, 2, 10)
    ans4 = [0.0620410301, 0.0875807131, 0.113451958, 0.139561671, 0.1657074530, 0.1908244840, 0.2070270720,
            0.207027072, 0.169718100, 0.0575152142, 0.00678695871] + [0] * 6 + \
        [0.000536304908, 0.0172181073, 0.041909870] + [0] * 10
    np.testing.assert_allclose(out4, ans4, rtol=1e-8, atol=0)


def test_smooth_sensitivity_conditions():
    assert ss.check_conditions(20, 10, 25.) == (True, False)
    assert ss.check_conditions(30, 10, 25.) == (True, True)


# ---------------------------------------------------------------- GPU kernels


@pytest.mark.gpu
def test_clip_sum_noise_gpu_matches_host():
    r = torch.Generator().manual_seed(0)
    for M, P in [(1, 5), (7, 1030), (256, 26010), (300, 40001)]:
        G = torch.randn(M, P, generator=r) * torch.rand(M, 1, generator=r) * 3
        host, hn = dpops.clip_sum_noise(G, 1.0, 1.12, M, seed=123, offset=7, return_norms=True)
        dev, dn = dpops.clip_sum_noise(G.cuda(), 1.0, 1.12, M, seed=123, offset=7, return_norms=True)
        torch.testing.assert_close(dn.cpu(), hn, rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dev.cpu(), host, rtol=1e-4, atol=2e-5)


@pytest.mark.gpu
def test_noisy_max_gpu_matches_host():
    r = np.random.default_rng(1)
    T, N, C = 250, 10007, 10
    labels = r.integers(0, C, (T, N)).astype(np.int32)
    for mode, scale in (("laplace", 20.0), ("gaussian", 40.0)):
        h, hv = dpops.noisy_max(labels, C, scale, mode, 9, 3, True)
        d, dv = dpops.noisy_max(labels, C, scale, mode, 9, 3, True, device="cuda")
        assert np.array_equal(hv, dv)
        assert (h == d).mean() > 0.999  # exact up to float ties from log/sincos ulps


@pytest.mark.gpu
def test_dp_sgd_mnist_cnn_gpu_step():
    from mifx.models.cnn import MnistDPCNN

    torch.manual_seed(0)
    m = MnistDPCNN().cuda()
    opt = DPGradientDescentOptimizer(1.0, 1.12, 256, m.parameters(), 0.08, seed=5)
    x = torch.randn(256, 28, 28, device="cuda")
    y = torch.randint(0, 10, (256,), device="cuda")
    loss = opt.step(m, lambda out, t: torch.nn.functional.cross_entropy(out, t, reduction="none"), x, y)
    assert math.isfinite(loss) and opt.last_norms.shape == (256,)


def _vmap_microbatch_grads(model, x, y, M):
    """fp32 reference: torch.func per-microbatch gradients of the summed CE loss, [M, P] in parameter order."""
    from torch.func import functional_call, grad, vmap

    params = {n: p.detach() for n, p in model.named_parameters()}

    def f(p, xb, yb):
        return torch.nn.functional.cross_entropy(functional_call(model, p, (xb,)), yb, reduction="sum")

    g = vmap(grad(f), in_dims=(None, 0, 0))(params, x.reshape(M, -1, *x.shape[1:]), y.reshape(M, -1))
    return torch.cat([g[n].reshape(M, -1) for n in params], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("B,M", [(64, 64), (64, 16), (96, 1)])
def test_dpsgd_mnist_fused_grads_match_vmap(B, M):
    """csrc/dpsgd_mnist.hip: whole-network per-microbatch gradients == vmap(grad) of the torch model (fp32)."""
    from mifx.models.cnn import MnistDPCNN
    from mifx.ops import dpsgd_mnist

    torch.manual_seed(1)
    m = MnistDPCNN().cuda()
    x = torch.rand(B, 28, 28, device="cuda")
    y = torch.randint(0, 10, (B,), device="cuda")
    y[3] = -100  # ignored label: zero loss and gradient, as F.cross_entropy
    G, loss = dpsgd_mnist.per_microbatch_grads(m, x, y, M)
    torch.cuda.synchronize()
    assert G.shape == (M, dpsgd_mnist.LD) and bool((G[:, dpsgd_mnist.NUM_PARAMS:] == 0).all())
    ref = _vmap_microbatch_grads(m, x, y, M)
    scale = ref.abs().amax(1, keepdim=True).clamp_min(1e-6)  # (row of the ignored label is all zero)
    torch.testing.assert_close(G[:, :dpsgd_mnist.NUM_PARAMS] / scale, ref / scale, rtol=0, atol=2e-5)
    ref_loss = torch.nn.functional.cross_entropy(m(x), y, reduction="none")
    torch.testing.assert_close(loss, ref_loss, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_dpsgd_mnist_fused_step_matches_generic_path():
    """The DP optimizer's fused MNIST path (sparse_softmax_ce) and its generic vmap path take the same step
    (same clip, same Philox noise stream)."""
    from mifx.models.cnn import MnistDPCNN
    from mifx.privacy import sparse_softmax_ce

    torch.manual_seed(2)
    ma = MnistDPCNN().cuda()
    mb = MnistDPCNN().cuda()
    mb.load_state_dict(ma.state_dict())
    oa = DPGradientDescentOptimizer(1.0, 1.12, 32, ma.parameters(), 0.08, seed=7)
    ob = DPGradientDescentOptimizer(1.0, 1.12, 32, mb.parameters(), 0.08, seed=7)
    for it in range(3):
        x = torch.rand(128, 28, 28, device="cuda")
        y = torch.randint(0, 10, (128,), device="cuda")
        la = float(oa.step(ma, sparse_softmax_ce, x, y))
        lb = float(ob.step(mb, lambda out, t: torch.nn.functional.cross_entropy(out, t, reduction="none"), x, y))
        assert abs(la - lb) < 1e-4 * max(1.0, abs(lb))
        torch.testing.assert_close(oa.last_norms, ob.last_norms, rtol=1e-4, atol=1e-6)
    for (n, pa), pb in zip(ma.named_parameters(), mb.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-4, atol=1e-5, msg=n)


# ---------------------------------------------------------------- more query / optimizer behaviour
# (reference: gaussian_query_test.py test_incompatible_records, nested_query_test.py test_complex_nested_query /
#  test_nested_query_with_noise, no_privacy_query_test.py, dp_optimizer_test.py testEstimator)


@pytest.mark.parametrize("query", [Q.GaussianSumQuery(10.0, 0.0), Q.NoPrivacySumQuery(),
                                   Q.GaussianAverageQuery(10.0, 0.0, 1.0), Q.NoPrivacyAverageQuery()])
@pytest.mark.parametrize("rec1,rec2", [
    (torch.zeros(2), torch.zeros(3)),                       # shape mismatch
    ([torch.zeros(2), torch.zeros(1)], [torch.zeros(2)]),   # structure mismatch
])
def test_incompatible_records_raise(query, rec1, rec2):
    with pytest.raises((ValueError, TypeError, RuntimeError)):
        _run_query(query, [rec1, rec2])


def test_no_privacy_sum_and_average_exact():
    r = [torch.tensor([1.0, 2.0]), torch.tensor([3.0, 5.0]), torch.tensor([-1.0, 2.0])]
    s, _ = _run_query(Q.NoPrivacySumQuery(), r)
    a, _ = _run_query(Q.NoPrivacyAverageQuery(), r)
    torch.testing.assert_close(s, torch.tensor([3.0, 9.0]))
    torch.testing.assert_close(a, torch.tensor([1.0, 3.0]))


def test_complex_nested_query():
    """Sums and averages at several nesting depths, each clipping its own sub-record."""
    q = Q.NestedQuery({"a": Q.GaussianSumQuery(1.0, 0.0),
                       "b": [Q.GaussianAverageQuery(10.0, 0.0, 2.0), (Q.NoPrivacySumQuery(),
                                                                      Q.GaussianSumQuery(5.0, 0.0))]})
    recs = [{"a": torch.tensor([3.0, 4.0]), "b": [torch.tensor([2.0]), (torch.tensor([1.0]), torch.tensor([6.0, 8.0]))]},
            {"a": torch.tensor([0.3, 0.4]), "b": [torch.tensor([4.0]), (torch.tensor([2.0]), torch.tensor([0.0, 1.0]))]}]
    out, _ = _run_query(q, recs)
    torch.testing.assert_close(out["a"], torch.tensor([0.6 + 0.3, 0.8 + 0.4]))   # first record clipped to norm 1
    torch.testing.assert_close(out["b"][0], torch.tensor([3.0]))                  # (2 + 4) / 2
    torch.testing.assert_close(out["b"][1][0], torch.tensor([3.0]))
    torch.testing.assert_close(out["b"][1][1], torch.tensor([3.0, 5.0]))          # [6,8] clipped to [3,4] + [0,1]


def test_nested_query_noise_std_per_leaf():
    g = torch.Generator().manual_seed(7)
    q = Q.NestedQuery([Q.GaussianSumQuery(1.0, 1.0, generator=g), Q.GaussianSumQuery(1.0, 3.0, generator=g)])
    draws = np.array([[float(x) for x in _run_query(q, [[torch.zeros(1), torch.zeros(1)]])[0]] for _ in range(1500)])
    assert draws[:, 0].std() == pytest.approx(1.0, abs=0.1)
    assert draws[:, 1].std() == pytest.approx(3.0, abs=0.25)


def test_make_optimizer_class_wraps_any_torch_optimizer():
    from mifx.privacy.optimizers import make_optimizer_class

    DPRMSprop = make_optimizer_class(torch.optim.RMSprop)
    assert DPRMSprop.__name__ == "DPRMSpropOptimizer"
    model = _Var([1.0, 2.0])
    opt = DPRMSprop(l2_norm_clip=1.0e9, noise_multiplier=0.0, num_microbatches=2, params=model.parameters(),
                    learning_rate=0.01)
    opt.compute_gradients(model, _half_sq, torch.tensor([[3.0, 4.0], [5.0, 6.0]]), torch.zeros(2))
    torch.testing.assert_close(model.v.grad, torch.tensor([-3.0, -3.0]))
    with pytest.raises(TypeError):
        make_optimizer_class(42)


def test_dp_sgd_linear_regression_converges():
    """The reference's estimator integration test: DP-SGD with clipping + noise fits y = X w* + b*."""
    g = torch.Generator().manual_seed(0)
    X = torch.randn(2000, 4, generator=g)
    w_true, b_true = torch.tensor([-6.0, -3.0, 2.0, 5.0]), 1.0
    y = X @ w_true + b_true
    model = torch.nn.Linear(4, 1)
    opt = DPGradientDescentOptimizer(l2_norm_clip=100.0, noise_multiplier=0.1, num_microbatches=20,
                                     params=model.parameters(), learning_rate=0.5, seed=5)
    for step in range(150):
        i = torch.randint(0, 2000, (20,), generator=g)
        opt.step(model, lambda out, t: 0.5 * (out.squeeze(-1) - t) ** 2, X[i], y[i])
    torch.testing.assert_close(model.weight.detach().squeeze(0), w_true, atol=1.0, rtol=0)
    assert abs(float(model.bias) - b_true) < 1.0


@pytest.mark.gpu
def test_mnist_fused_mean_grads_match_autograd():
    """Non-private step on the per-example kernel: p.grad == autograd of the mean cross-entropy (fp32)."""
    from mifx.models.cnn import MnistDPCNN
    from mifx.ops import dpsgd_mnist

    torch.manual_seed(3)
    m = MnistDPCNN().cuda()
    x = torch.rand(48, 28, 28, device="cuda")
    y = torch.randint(0, 10, (48,), device="cuda")
    loss = dpsgd_mnist.assign_mean_grads(m, x, y)
    got = [p.grad.clone() for p in m.parameters()]
    m.zero_grad()
    ref_loss = torch.nn.functional.cross_entropy(m(x), y)
    ref_loss.backward()
    assert abs(float(loss) - float(ref_loss)) < 1e-5
    for g, p in zip(got, m.parameters()):
        s = p.grad.abs().max().clamp_min(1e-8)
        torch.testing.assert_close(g / s, p.grad / s, rtol=0, atol=2e-5)


def test_rdp_gaussian_theorem6_direct_evaluation():
    """Own goldens for the GNMax data-dependent bound (Theorem 6): at moderate q the log-space implementation must
    equal the theorem's formula evaluated directly, stay below the data-independent lambda / sigma^2, and grow
    with q."""
    import math

    import numpy as np

    from mifx.privacy.pate import rdp2018 as core

    sigma = 40.0
    lam = np.array([2.0, 5.0, 10.0, 20.0])
    prev = None
    for q in (1e-6, 1e-5, 1e-4):
        got = core.rdp_gaussian(math.log(q), sigma, lam)
        mu2 = math.sqrt(sigma ** 2 * math.log(1 / q))
        mu1 = mu2 + 1
        e1, e2 = mu1 / sigma ** 2, mu2 / sigma ** 2
        A = (1 - q) / (1 - (q * math.exp(e2)) ** ((mu2 - 1) / mu2))
        B = math.exp(e1) / q ** (1 / (mu1 - 1))
        direct = np.log((1 - q) * A ** (lam - 1) + q * B ** (lam - 1)) / (lam - 1)
        want = np.where(lam < mu1, np.minimum(lam / sigma ** 2, direct), lam / sigma ** 2)
        np.testing.assert_allclose(got, want, rtol=1e-8, atol=1e-15)
        assert np.all(got <= lam / sigma ** 2 + 1e-15)
        if prev is not None:
            assert np.all(got >= prev - 1e-15)
        prev = got
    assert core.rdp_gaussian(-math.inf, sigma, 7.0) == 0.0


def test_smooth_sensitivity_threshold_low_threshold_golden():
    """`smooth_sensitivity_test.py:82-92` (t = 2, below every count)."""
    c = np.array([20, 10, 0])
    out2 = ss.compute_local_sensitivity_bounds_threshold(c, int(c.sum()), 2, 2, 10)
    ans2 = [1.60212079e-01, 2.07021132e-01, 2.07021132e-01, 1.93127860e-01, 1.68302106e-01, 1.42180452e-01,
            1.16054002e-01, 9.01543247e-02, 6.45775697e-02, 3.94153241e-02, 1.47826870e-02, 1.48454129e-04] + [0] * 18
    np.testing.assert_allclose(out2, ans2, rtol=5e-8, atol=0)


def test_pate2017_sensitivity_uses_sorted_counts():
    """The distance-k check uses the plurality and runner-up of the SORTED counts (the reference compared the
    unsorted input's first two entries): permuting the classes does not change the smooth sensitivity."""
    c = np.array([3, 200, 40, 7])
    perm = np.array([200, 40, 7, 3])
    for l in (1.0, 4.0):
        assert analysis2017.smoothed_sens(c, 0.05, l, 0.09) == analysis2017.smoothed_sens(perm, 0.05, l, 0.09)
        assert analysis2017.smoothed_sens(perm, 0.05, l, 0.09) > 0
