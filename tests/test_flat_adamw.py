"""Flat mixed-precision AdamW (csrc/adamw.hip) vs torch.optim.AdamW / the CPU reference."""
import pytest
import torch

from mifx.ops.adamw import adamw_flat_
from mifx.trainer.optim import FlatAdamW


def test_flat_adamw_cpu_matches_torch_adamw():
    torch.manual_seed(0)
    m1 = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 3))
    m2 = torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.Linear(7, 3))
    m2.load_state_dict(m1.state_dict())
    ref = torch.optim.AdamW(m1.parameters(), lr=1e-2, weight_decay=0.01)
    opt = FlatAdamW(m2.parameters(), lr=1e-2, weight_decay=0.01, dtype=torch.float32)
    x = torch.randn(16, 5)
    for _ in range(5):
        ref.zero_grad()
        m1(x).pow(2).sum().backward()
        ref.step()
        opt.zero_grad()
        m2(x).pow(2).sum().backward()
        opt.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    assert int(opt.step_count) == 5


@pytest.mark.gpu
def test_flat_adamw_kernel_matches_reference():
    torch.manual_seed(0)
    n = 8 * 1000 + 5  # vector body + scalar tail
    master = torch.randn(n)
    g = (torch.randn(n) * 0.1).bfloat16()
    bufs_cpu = [master.bfloat16(), g, master.clone(), torch.zeros(n), torch.zeros(n), torch.zeros((), dtype=torch.int32)]
    bufs_gpu = [t.cuda() for t in bufs_cpu]
    for _ in range(3):
        adamw_flat_(*bufs_cpu, lr=1e-3, weight_decay=0.01)
        adamw_flat_(*bufs_gpu, lr=1e-3, weight_decay=0.01)
    for a, b in zip(bufs_cpu[2:5], bufs_gpu[2:5]):
        torch.testing.assert_close(b.cpu(), a, rtol=1e-5, atol=1e-6)
    assert torch.equal(bufs_gpu[0].cpu(), bufs_gpu[2].cpu().bfloat16())
    assert int(bufs_gpu[5]) == 3


@pytest.mark.gpu
def test_flat_adamw_own_grads_matches_views_mode():
    """grads='own' (chunked kernel reading autograd's per-parameter gradients in place, no zero-fill / no
    accumulate kernels) must give the same update as grads='views' (flat gradient buffer); a parameter
    without a gradient is left untouched (torch AdamW semantics). Odd sizes exercise the 8-aligned
    flat offsets and the scalar tails; a 20000-wide layer spans several 8192-element chunks."""
    torch.manual_seed(0)

    def make():
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.GELU(), torch.nn.Linear(7, 20000),
                                   torch.nn.Linear(20000, 3)).cuda().bfloat16()

    ma, mb = make(), make()
    unused = torch.nn.Parameter(torch.randn(13, device="cuda", dtype=torch.bfloat16))
    before = unused.detach().clone()
    oa = FlatAdamW(list(ma.parameters()), lr=1e-3, weight_decay=0.01, grads="views")
    ob = FlatAdamW(list(mb.parameters()) + [unused], lr=1e-3, weight_decay=0.01, grads="own")
    x = torch.randn(64, 5, device="cuda", dtype=torch.bfloat16)
    for _ in range(4):
        for m, o in ((ma, oa), (mb, ob)):
            o.zero_grad()
            m(x).float().pow(2).mean().backward()
            o.step()
    torch.cuda.synchronize()
    for a, b in zip(ma.parameters(), mb.parameters()):
        torch.testing.assert_close(b.float(), a.float(), rtol=0, atol=0)
    assert torch.equal(unused.detach(), before)
    assert int(ob.step_count) == 4 and all(p.grad is not None for p in mb.parameters())
    ob.zero_grad()
    assert all(p.grad is None for p in mb.parameters())


@pytest.mark.gpu
def test_overlapped_bucket_update_in_captured_step_is_bit_identical():
    """grads='own' with overlap: in a captured step each parameter bucket's update is launched on a side stream from
    the post-accumulate-grad hook of its last gradient (under the rest of the backward), the step counter advanced
    once at the end. After graph replays the weights must equal the single-launch update bit for bit; an unused
    parameter (never gets a gradient) is left untouched."""
    def make():
        torch.manual_seed(1)
        return torch.nn.Sequential(torch.nn.Linear(5, 7), torch.nn.GELU(), torch.nn.Linear(7, 20000),
                                   torch.nn.Linear(20000, 3), torch.nn.Linear(3, 9)).cuda().bfloat16()

    x = torch.randn(64, 5, device="cuda", dtype=torch.bfloat16)
    out = []
    for overlap in (False, True):
        m = make()
        unused = torch.nn.Parameter(torch.ones(13, device="cuda", dtype=torch.bfloat16))
        o = FlatAdamW(list(m.parameters()) + [unused], lr=1e-3, weight_decay=0.01, grads="own", overlap=overlap,
                      bucket_elems=4096)  # several buckets of whole parameters
        if overlap:
            assert len(o._buckets) > 2

        def step():
            o.zero_grad()
            m(x).float().pow(2).mean().backward()
            o.step()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):
                step()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        o.zero_grad()
        o.begin_capture()
        with torch.cuda.graph(g):
            step()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        assert int(o.step_count) == 2 + 5  # (capturing records the step, it does not run it)
        assert torch.equal(unused.detach(), torch.ones_like(unused))
        out.append(o.flat.clone())
    assert torch.equal(out[0], out[1])
