"""Fused multi-tensor SGD (csrc/sgd.hip) against torch.optim.SGD's foreach update (mifx.ops.sgd.sgd_reference_):
weight decay per tensor, momentum, dampening, Nesterov, learning rate from a device tensor; odd tensor sizes
(unvectorised tails, chunk boundaries)."""
import pytest
import torch



def test_dense_layout_check_cpu():
    from mifx.ops.sgd import _dense

    assert _dense(torch.randn(64, 32, 3, 3).contiguous(memory_format=torch.channels_last))
    assert _dense(torch.randn(5, 7).t()) and _dense(torch.randn(3, 1, 4))
    assert not _dense(torch.randn(5, 7)[:, :3]) and not _dense(torch.randn(8)[::2])


@pytest.mark.gpu
@pytest.mark.parametrize("nesterov,damp", [(True, 0.0), (False, 0.0), (False, 0.1)])
def test_fused_sgd_matches_foreach(nesterov, damp):
    from mifx.ops.sgd import FusedSGDTables, sgd_reference_

    torch.manual_seed(0)
    sizes = [7, 64, 1000, 2048, 2048 * 3 + 5, 4096 + 3]
    wds = [1e-4 if i % 2 else 0.0 for i in range(len(sizes))]
    mk = lambda: [torch.randn(n, device="cuda") for n in sizes]  # noqa: E731
    params, grads, bufs = mk(), mk(), mk()
    p2, g2, b2 = ([t.clone() for t in ts] for ts in (params, grads, bufs))
    neg_lr = torch.tensor(-0.05, device="cuda")
    tab = FusedSGDTables(params, bufs, wds, grads=grads)
    assert tab.matches(params, bufs)
    for _ in range(3):
        tab.step(neg_lr, 0.9, damp, nesterov)
        for i, w in enumerate(wds):  # the reference per weight-decay value, as torch's param groups do
            sgd_reference_([p2[i]], [g2[i]], [b2[i]], w, 0.9, damp, nesterov, neg_lr)
    for a, b in zip(params + bufs, p2 + b2):
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6)
    assert all(torch.equal(g, h) for g, h in zip(grads, g2))  # gradients are read only


@pytest.mark.gpu
def test_fused_sgd_channels_last_tensors():
    """channels_last convolution weights (dense, not contiguous): the flat update equals the reference; a layout
    mismatch between a parameter and its gradient is refused."""
    from mifx.ops.sgd import FusedSGDTables, sgd_reference_

    torch.manual_seed(2)
    cl = lambda: torch.randn(64, 32, 3, 3, device="cuda").contiguous(memory_format=torch.channels_last)  # noqa: E731
    p, g, b = [cl()], [cl()], [cl()]
    ref = [p[0].clone()], [b[0].clone()]
    neg_lr = torch.tensor(-0.1, device="cuda")
    FusedSGDTables(p, b, [5e-5], grads=g).step(neg_lr, 0.9, 0.0, True)
    sgd_reference_(ref[0], g, ref[1], 5e-5, 0.9, 0.0, True, neg_lr)
    torch.testing.assert_close(p[0], ref[0][0], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(b[0], ref[1][0], rtol=1e-6, atol=1e-6)
    with pytest.raises(ValueError):
        FusedSGDTables(p, b, [0.0], grads=[g[0].contiguous()])


@pytest.mark.gpu
def test_fused_sgd_in_captured_graph_follows_device_lr():
    from mifx.ops.sgd import FusedSGDTables, sgd_reference_

    torch.manual_seed(1)
    p = [torch.randn(3000, device="cuda")]
    g = [torch.randn(3000, device="cuda")]
    b = [torch.zeros(3000, device="cuda")]
    ref = [t.clone() for t in p], [t.clone() for t in b]
    neg_lr = torch.tensor(-0.1, device="cuda")
    tab = FusedSGDTables(p, b, [1e-4])
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            tab.set_grads(g)  # the address copy is a graph node
            tab.step(neg_lr, 0.9, 0.0, True)
    torch.cuda.current_stream().wait_stream(s)
    for lr in (0.1, 0.2, 0.05):
        neg_lr.fill_(-lr)
        graph.replay()
        sgd_reference_(ref[0], g, ref[1], 1e-4, 0.9, 0.0, True, torch.tensor(-lr, device="cuda"))
    torch.cuda.synchronize()
    torch.testing.assert_close(p[0], ref[0][0], rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(b[0], ref[1][0], rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
def test_fused_sgd_capture_keeps_addresses_and_invalidates_weight_images():
    """(1) A set_grads after a capture does not retarget the captured graph (each capture owns its address buffer).
    (2) The update bumps the parameters' version counters, so the bf16 weight images refreshed before it are stale:
    an eager conv forward after the captured step equals F.conv2d with the CURRENT weights."""
    import torch.nn.functional as F

    from mifx.ops import conv1x1
    from mifx.ops.sgd import FusedSGDTables
    from mifx.ops.weight_prep import WeightPrep, images

    torch.manual_seed(3)
    w = torch.randn(128, 64, 1, 1, device="cuda") * 0.1
    b = torch.zeros_like(w)
    g = [torch.randn_like(w)]
    other = [torch.randn_like(w) * 100]
    prep = WeightPrep([w])
    neg_lr = torch.tensor(-0.5, device="cuda")
    tab = FusedSGDTables([w], [b], [0.0])
    with pytest.raises(RuntimeError):
        tab.step(neg_lr, 0.9, 0.0, False)  # no gradients yet
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            prep.refresh()
            tab.set_grads(g)
            tab.step(neg_lr, 0.9, 0.0, False)
    torch.cuda.current_stream().wait_stream(s)
    tab.set_grads(other)  # eager retarget: must not leak into the graph
    w0 = w.clone()
    graph.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(w, w0 - 0.5 * g[0], rtol=1e-6, atol=1e-6)  # momentum buffer was zero
    assert images(w) is None  # the images predate the update
    x = torch.randn(4, 64, 16, 16, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    assert conv1x1.eligible(x, w)
    y = conv1x1.conv1x1(x, w)[0]
    ref = F.conv2d(x.float(), w.float())
    torch.testing.assert_close(y.float(), ref, rtol=3e-2, atol=3e-2)
    stale = F.conv2d(x.float(), w0.float())
    assert (y.float() - stale).abs().max() > 10 * (y.float() - ref).abs().max()  # the update is visible
    prep.close()
