"""Fashion-MNIST train -> versioned export -> REST serving (reference
`notebooks/serving/Predict_Fashion_MNIST.ipynb` cells 8-31): Conv(8, 3x3, s2) + Dense(10, softmax),
5 epochs of Adam, export to <model_dir>/<version>, inspect the signature (saved_model_cli
equivalent), start the model server (`mifx-model-server --rest_api_port 8501 --model_name
fashion_model --model_base_path <model_dir>`) and query
`POST /v1/models/fashion_model:predict` and `/v1/models/fashion_model/versions/1:predict` with
`{"signature_name": "serving_default", "instances": [...]}`. Synthetic Fashion-MNIST-shaped data
(no downloads offline)."""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import requests  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from mifx.data.synthetic import synthetic_images  # noqa: E402
from mifx.models.cnn import FashionCNN  # noqa: E402
from mifx.serving.saved_model import save_module  # noqa: E402

CLASS_NAMES = ["T-shirt/top", "Trouser", "Pullover", "Dress", "Coat", "Sandal", "Shirt", "Sneaker", "Bag",
               "Ankle boot"]


def train(x, y, epochs: int = 5, batch: int = 32, device="cpu") -> FashionCNN:
    torch.manual_seed(0)
    m = FashionCNN().to(device)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    x, y = x.to(device), y.to(device)
    for ep in range(epochs):
        perm = torch.randperm(len(x), device=device)
        tot = 0.0
        for i in range(0, len(x), batch):
            idx = perm[i:i + batch]
            opt.zero_grad()
            loss = F.cross_entropy(m.logits(x[idx]), y[idx])
            loss.backward()
            opt.step()
            tot += float(loss.detach()) * len(idx)
        print(f"epoch {ep + 1}/{epochs} loss {tot / len(x):.4f}")
    return m.cpu().eval()


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model_dir", default=os.path.join(tempfile.gettempdir(), "fashion_model"))
    ap.add_argument("--train_size", type=int, default=60000)
    ap.add_argument("--epochs", type=int, default=5)
    ap.add_argument("--version", type=int, default=1)
    ap.add_argument("--port", type=int, default=0, help="REST port (0: pick a free one; the notebook uses 8501)")
    a = ap.parse_args(argv)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    x, y = synthetic_images(a.train_size + 1000, seed=5)
    xtr, ytr, xte, yte = x[:a.train_size], y[:a.train_size], x[a.train_size:], y[a.train_size:]
    model = train(xtr, ytr, a.epochs, device=dev)
    with torch.no_grad():
        acc = float((model(xte).argmax(1) == yte).float().mean())
    print(f"Test accuracy: {acc:.4f}")
    export_path = os.path.join(a.model_dir, str(a.version))
    save_module(export_path, model, "mifx.models.cnn:FashionCNN", {}, [28, 28], class_names=CLASS_NAMES)
    with open(os.path.join(export_path, "saved_model.json")) as f:
        print("signature_def['serving_default']:", json.dumps(json.load(f)["signatures"]["serving_default"]))

    port = a.port or _free_port()
    srv = subprocess.Popen([sys.executable, "-m", "mifx.serving.server", "--rest_api_port", str(port),
                            "--model_name", "fashion_model", "--model_base_path", a.model_dir, "--device", "cpu"],
                           cwd=os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
    try:
        url = f"http://127.0.0.1:{port}/v1/models/fashion_model"
        for _ in range(200):
            try:
                if requests.get(url, timeout=1).status_code == 200:
                    break
            except requests.ConnectionError:
                time.sleep(0.1)
        data = json.dumps({"signature_name": "serving_default", "instances": xte[:3].numpy().tolist()})
        headers = {"content-type": "application/json"}
        latest = requests.post(url + ":predict", data=data, headers=headers).json()["predictions"]
        pinned = requests.post(url + f"/versions/{a.version}:predict", data=data, headers=headers).json()["predictions"]
        for i, p in enumerate(latest):
            print(f"The model thought this was a {CLASS_NAMES[int(np.argmax(p))]} (class {int(np.argmax(p))}), "
                  f"and it was actually a {CLASS_NAMES[int(yte[i])]} (class {int(yte[i])})")
    finally:
        srv.terminate()
        srv.wait(timeout=30)
    return {"accuracy": acc, "latest": latest, "pinned": pinned, "labels": yte[:3].tolist()}


if __name__ == "__main__":
    main()
