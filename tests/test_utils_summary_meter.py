"""TensorBoard-compatible summaries, examples/sec meter, fairing MNIST example."""
import importlib.util
import os
import struct

from mifx.io.tfrecord import masked_crc32c
from mifx.utils import ExamplesPerSec, SummaryWriter, read_scalars, trace_range


def test_summary_roundtrip_and_framing(tmp_path):
    with SummaryWriter(str(tmp_path)) as w:
        for s in range(5):
            w.add_scalar("loss", 1.0 / (s + 1), s * 100)
        w.add_scalar("lr", 0.3, 0)
    sc = read_scalars(str(tmp_path))
    assert [s for s, _ in sc["loss"]] == [0, 100, 200, 300, 400]
    assert abs(sc["loss"][1][1] - 0.5) < 1e-7 and sc["lr"] == [(0, 0.30000001192092896)]
    raw = open(w.path, "rb").read()
    (n,) = struct.unpack("<Q", raw[:8])
    assert struct.unpack("<I", raw[8:12])[0] == masked_crc32c(raw[:8])
    assert b"brain.Event:2" in raw[12:12 + n]  # file_version record first, as TensorBoard expects


def test_examples_per_sec_meter_logs_every_n():
    lines = []
    m = ExamplesPerSec(batch_size=128, every=10, device="cpu", log=lines.append)
    for step in range(25):
        with trace_range("step"):
            m.step(step, loss=0.5)
    assert len(m.history) == 3 and m.history[1]["step"] == 10
    assert "examples/sec" in lines[0] and m.history[-1]["examples_per_sec"] > 0


def test_fairing_mnist_model_trains_and_writes_summaries(tmp_path):
    p = os.path.join(os.path.dirname(__file__), "..", "examples", "fairing", "fairing_mnist.py")
    spec = importlib.util.spec_from_file_location("fairing_mnist", p)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    res = mod.TorchMnistModel(max_steps=300, log_dir=str(tmp_path)).train()
    assert res["losses"][-1] < res["losses"][0]
    assert [s for s, _ in read_scalars(str(tmp_path))["loss"]] == [0, 100, 200]
