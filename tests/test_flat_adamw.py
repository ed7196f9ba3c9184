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
