"""Smoke runs of the privacy examples at toy sizes (CPU)."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(__file__))


def _load(rel):
    spec = importlib.util.spec_from_file_location(rel.replace("/", "_"), os.path.join(ROOT, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_mnist_dpsgd_example():
    acc = _load("examples/privacy/mnist_dpsgd.py").main(["--epochs", "1", "--train_size", "1024", "--device", "cpu",
                                                         "--batch_size", "64", "--microbatches", "16"])
    assert 0.0 <= acc <= 1.0


def test_pate_example():
    acc, rep = _load("examples/privacy/pate_mnist.py").main(
        ["--nb_teachers", "2", "--teacher_steps", "5", "--student_steps", "5", "--stdnt_share", "100",
         "--train_size", "800", "--device", "cpu"])
    assert 0.0 <= acc <= 1.0 and rep["eps"] > 0
