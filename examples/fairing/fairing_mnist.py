"""Remote MNIST training through the fairing-style config (reference
`kubeflow-pipelines/fairing/fairing_tf.py:40-80`): a model object whose `train()` runs a feed-style
loop (2000 steps, batch 100, two hidden layers 128/32, SGD lr 0.3 as the TF `mnist.training` op),
printing the loss and writing a `loss` scalar summary every 100 steps to a TensorBoard-readable
log dir; `fairing.config.set_model(model); fairing.config.run()` executes it in a separate
process (deployer "local") or as a Kubernetes Job on AMD GPUs (deployer "job").
MNIST is synthetic offline (same 784-pixel shape)."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

MAX_STEPS, BATCH_SIZE, LEARNING_RATE, HIDDEN_1, HIDDEN_2 = 2000, 100, 0.3, 128, 32
LOG_DIR = os.path.join(os.getenv("TEST_TMPDIR", "/tmp"), "mifx/mnist/logs/fully_connected_feed/",
                       os.getenv("HOSTNAME", ""))


class TorchMnistModel:
    def __init__(self, max_steps: int = MAX_STEPS, log_dir: str = LOG_DIR):
        self.max_steps, self.log_dir = max_steps, log_dir

    def train(self, **kwargs):
        import torch
        import torch.nn.functional as F

        from mifx.data.synthetic import synthetic_images
        from mifx.utils import SummaryWriter

        dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        x, y = synthetic_images(55000, seed=2)
        x = x * (x > 0.7)  # MNIST-like sparse strokes (~13% mean intensity) for the lr-0.3 SGD recipe
        x, y = x.reshape(len(x), 784).to(dev), y.to(dev)
        torch.manual_seed(0)
        model = torch.nn.Sequential(torch.nn.Linear(784, HIDDEN_1), torch.nn.ReLU(),
                                    torch.nn.Linear(HIDDEN_1, HIDDEN_2), torch.nn.ReLU(),
                                    torch.nn.Linear(HIDDEN_2, 10)).to(dev)
        for m in model:  # tf mnist.inference: truncated normal(stddev 1/sqrt(fan_in)), zero biases
            if isinstance(m, torch.nn.Linear):
                torch.nn.init.trunc_normal_(m.weight, std=1.0 / m.in_features ** 0.5, a=-2.0 / m.in_features ** 0.5,
                                            b=2.0 / m.in_features ** 0.5)
                torch.nn.init.zeros_(m.bias)
        opt = torch.optim.SGD(model.parameters(), lr=LEARNING_RATE)
        losses = []
        with SummaryWriter(self.log_dir) as writer:
            pos = 0
            for step in range(self.max_steps):
                if pos + BATCH_SIZE > len(x):  # next_batch(shuffle=False): wrap to the start
                    pos = 0
                xb, yb = x[pos:pos + BATCH_SIZE], y[pos:pos + BATCH_SIZE]
                pos += BATCH_SIZE
                opt.zero_grad(set_to_none=True)
                loss = F.cross_entropy(model(xb), yb)
                loss.backward()
                opt.step()
                if step % 100 == 0:
                    lv = float(loss.detach())
                    print("At step {}, loss = {}".format(step, lv))
                    writer.add_scalar("loss", lv, step)
                    writer.flush()
                    losses.append(lv)
        return {"losses": losses, "log_dir": self.log_dir}


if __name__ == "__main__":
    from mifx import fairing

    fairing.config.set_builder("append", base_image="rocm/pytorch:latest", registry="local", push=False)
    fairing.config.set_deployer("local")
    fairing.config.set_model(TorchMnistModel())
    print(fairing.config.run())
