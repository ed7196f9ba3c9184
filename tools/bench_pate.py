"""PATE-2017 teacher training throughput: the reference's one-teacher-at-a-time recipe (`deep_cnn.train`, one
3000-step run per teacher) vs all teachers as one grouped network (`ensemble.train_ensemble`). MNIST shapes,
B=128 per teacher, shard = 60000/nb_teachers. Reports steady-state ms per step and teacher-steps per second
(one teacher-step = one SGD step of one teacher on its 128-example batch)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mifx.privacy.pate import deep_cnn, ensemble  # noqa: E402


def run(T, steps, dev, deeper=False):
    cfg = deep_cnn.DeepCNNConfig(max_steps=steps, batch_size=128, nb_teachers=T, deeper=deeper, log_every=10 ** 9,
                                 ckpt_every=10 ** 9)
    n = 60000 // T
    x, y, _, _ = deep_cnn.load_dataset("mnist", train_size=n * T, test_size=16)
    shards = [deep_cnn.partition_dataset(x, y, T, t) for t in range(T)]
    times = []
    ensemble.train_ensemble([s[0] for s in shards], [s[1] for s in shards], ["/tmp/unused"] * T, cfg, device=dev,
                            log=lambda *_: None, checkpoint=False, step_times=times)
    ms = 1e3 * float(np.median(times[3:]))
    return {"mode": "ensemble", "teachers": T, "deeper": deeper, "ms_per_step": ms,
            "teacher_steps_per_sec": T * 1e3 / ms, "examples_per_sec": T * 128 * 1e3 / ms,
            "est_3000_step_run_s": 3000 * ms / 1e3}


def run_sequential(steps, dev, deeper=False):
    """One teacher with deep_cnn.train's own loop; ms/step from total time (2 checkpoints included)."""
    cfg = deep_cnn.DeepCNNConfig(max_steps=steps, batch_size=128, nb_teachers=250, deeper=deeper,
                                 log_every=10 ** 9, ckpt_every=10 ** 9)
    x, y, _, _ = deep_cnn.load_dataset("mnist", train_size=60000, test_size=16)
    xs, ys = deep_cnn.partition_dataset(x, y, 250, 0)
    deep_cnn.train(xs, ys, "/tmp/pate_seq_bench.ckpt", cfg, device=dev, log=lambda *_: None)  # warm-up
    torch.cuda.synchronize()
    t0 = time.time()
    deep_cnn.train(xs, ys, "/tmp/pate_seq_bench.ckpt", cfg, device=dev, log=lambda *_: None)
    torch.cuda.synchronize()
    ms = 1e3 * (time.time() - t0) / steps
    return {"mode": "sequential", "teachers": 1, "deeper": deeper, "ms_per_step": ms,
            "teacher_steps_per_sec": 1e3 / ms, "examples_per_sec": 128e3 / ms,
            "est_250_teachers_3000_steps_s": 250 * 3000 * ms / 1e3}


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--teachers", default="10,50,250")
    ap.add_argument("--no-sequential", action="store_true")
    ap.add_argument("--deeper", action="store_true", help="inference_deeper (3x3 convs 96/192)")
    a = ap.parse_args()
    dev = "cuda"
    if not a.no_sequential:
        print(json.dumps(run_sequential(a.steps, dev, a.deeper)), flush=True)
    for T in [int(t) for t in a.teachers.split(",")]:
        print(json.dumps(run(T, a.steps, dev, a.deeper)), flush=True)
