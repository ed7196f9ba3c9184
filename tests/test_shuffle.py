"""Per-epoch record shuffling (csrc/feed.h, mifx.data.shuffle): the reference reads its training data with
`read_batch_features(randomize_input=True)` (`airflow-dags/taxi_utils.py:275-276`). An epoch must visit every
record exactly once, in an order fixed by (seed, epoch); the host implementation must be bit-exact to the kernels'
header; the GPU trainers must train on exactly the records the host implementation names."""
import os
import subprocess

import numpy as np
import pytest
import torch

from mifx.data import shuffle as sh

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 100, 1000, 4097, 15000])
@pytest.mark.parametrize("key", [1, 0x5EED, 2**63 + 12345])
def test_feistel_is_a_bijection(n, key):
    p = sh.feistel_perm(np.arange(n), n, sh.epoch_key(key, 3))
    assert np.array_equal(np.sort(p), np.arange(n))


@pytest.mark.parametrize("batch,n", [(40, 15000), (40, 1000), (7, 100), (64, 64)])
def test_epoch_visits_every_record_once_in_a_seed_determined_order(batch, n):
    steps = -(-2 * n // batch) + 1
    seq = np.concatenate([sh.record_indices(s, batch, n, seed=99) for s in range(steps)])
    e0, e1 = seq[:n], seq[n:2 * n]
    assert np.array_equal(np.sort(e0), np.arange(n)) and np.array_equal(np.sort(e1), np.arange(n))
    if n > 8:
        assert not np.array_equal(e0, e1), "every epoch draws a new order"
        assert not np.array_equal(e0, np.arange(n)), "shuffled"
    again = np.concatenate([sh.record_indices(s, batch, n, seed=99) for s in range(steps)])
    assert np.array_equal(seq, again)
    other = np.concatenate([sh.record_indices(s, batch, n, seed=98) for s in range(steps)])
    assert not np.array_equal(seq[:n], other[:n]) or n <= 2


def test_seed_zero_is_stored_order():
    got = np.concatenate([sh.record_indices(s, 40, 100) for s in range(5)])
    assert np.array_equal(got, np.arange(200) % 100)


def test_global_stream_slices_are_disjoint_and_equal_one_process():
    """World 4 x batch 10 with offsets rank x 10 reads the global batch of one process at batch 40, split."""
    n, B, W = 1234, 10, 4
    for step in (0, 5, 30, 31):
        parts = [sh.record_indices(step, B, n, W * B, r * B, seed=7) for r in range(W)]
        one = sh.record_indices(step, W * B, n, seed=7)
        assert np.array_equal(np.concatenate(parts), one)
        assert len(set(np.concatenate(parts).tolist())) == W * B


def test_host_implementation_bit_exact_to_kernel_header(tmp_path):
    """csrc/feed.h compiled for the host (g++) names the same records as mifx.data.shuffle."""
    src = tmp_path / "feedcheck.cpp"
    src.write_text(r'''
#include "feed.h"
#include <cstdio>
#include <cstdlib>
int main(int argc, char** argv) {
  long long n = atoll(argv[1]), batch = atoll(argv[2]), gs = atoll(argv[3]), go = atoll(argv[4]);
  unsigned long long key = strtoull(argv[5], 0, 10);
  long long steps = atoll(argv[6]);
  MifxFeed f{gs, go, key};
  for (long long s = 0; s < steps; ++s) {
    MifxFeedStep st = mifx_feed_step(f, s, n);
    for (long long r = 0; r < batch; ++r) printf("%lld\n", mifx_feed_record(f, st, r, n));
  }
  return 0;
}
''')
    exe = tmp_path / "feedcheck"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "csrc"), str(src), "-o", str(exe)],
                   check=True)
    for n, batch, gs, go, key, steps in [(15000, 40, 40, 0, 0x5EED, 400), (1000, 24, 96, 48, 2**64 - 3, 90),
                                         (97, 97, 97, 0, 1, 3), (1 << 20, 4096, 4096, 0, 12345, 4)]:
        out = subprocess.run([str(exe), str(n), str(batch), str(gs), str(go), str(key), str(steps)],
                             capture_output=True, text=True, check=True).stdout.split()
        got = np.array([int(x) for x in out])
        want = np.concatenate([sh.record_indices(s, batch, n, gs, go, key) for s in range(steps)])
        assert np.array_equal(got, want), (n, batch, key)


def test_cpu_wide_deep_trainer_trains_on_the_shuffled_records():
    """TorchWideDeepTrainer with a seed trains step s on record_indices(s): equal to an unshuffled trainer fed
    the permuted records explicitly."""
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.torch_wide_deep import TorchWideDeepTrainer

    recs = synthetic_records(300, device="cpu", seed=3)
    a = TorchWideDeepTrainer(wdm.WideDeepModel(seed=1), batch=40, shuffle_seed=11)
    a.set_data(recs)
    a.run(9)  # crosses the epoch boundary at step 7.5
    order = np.concatenate([sh.record_indices(s, 40, 300, seed=11) for s in range(9)])
    b = TorchWideDeepTrainer(wdm.WideDeepModel(seed=1), batch=40)
    b.set_data(recs[torch.from_numpy(order)])
    b.run(9)
    for (k, p), (_, q) in zip(a.model.named_parameters(), b.model.named_parameters()):
        torch.testing.assert_close(p, q, msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize("batch", [40, 4096])
def test_fused_wide_deep_kernel_fetches_the_shuffled_records(batch):
    """The fused kernel (csrc/wd_chain.hip fetch through csrc/feed.h) with a shuffle seed trains on exactly the
    records mifx.data.shuffle names: same weights as the kernel fed those records in stored order, across an
    epoch boundary (any wrong record would change the gradient)."""
    from mifx.data.synthetic import synthetic_records
    from mifx.models import wide_deep as wdm
    from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer

    n = batch * 5 + batch // 2
    steps = 8
    recs = synthetic_records(n, device="cuda", seed=5)
    a = FusedWideDeepTrainer(wdm.WideDeepModel(seed=2), batch=batch, device="cuda", shuffle_seed=0xC0FFEE)
    a.set_data(recs)
    for _ in range(steps):
        a.step()
    order = np.concatenate([sh.record_indices(s, batch, n, seed=0xC0FFEE) for s in range(steps)])
    b = FusedWideDeepTrainer(wdm.WideDeepModel(seed=2), batch=batch, device="cuda")
    b.set_data(recs[torch.from_numpy(order).cuda()])
    for _ in range(steps):
        b.step()
    torch.cuda.synchronize()
    assert torch.equal(a.param, b.param)


@pytest.mark.gpu
def test_taxi_dnn_gpu_shuffle_matches_cpu():
    """The taxi DNN kernels (csrc/embag_mlp.hip BatchSel through csrc/feed.h) and the CPU path pick the same
    shuffled records: weights agree after steps that cross an epoch."""
    from mifx.models.taxi_dnn import TaxiDNN, TaxiDNNConfig
    from mifx.trainer.taxi_dnn_trainer import TaxiDNNTrainer
    from tests.test_taxi_dnn import _data

    cfg = TaxiDNNConfig(hidden=96)
    ids, dense, y = _data(150, cfg, seed=4)
    cpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=6), batch=32, lr=0.1, device="cpu", shuffle_seed=77)
    gpu = TaxiDNNTrainer(TaxiDNN(cfg, seed=6), batch=32, lr=0.1, device="cuda", shuffle_seed=77, steps_per_graph=3)
    for tr in (cpu, gpu):
        tr.set_data(ids, dense, y)
        tr.run(11)
    for k in ("W1", "b1", "w2", "b2"):
        torch.testing.assert_close(getattr(gpu.model, k).detach().cpu(), getattr(cpu.model, k).detach(),
                                   rtol=2e-4, atol=2e-5)
