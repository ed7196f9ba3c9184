"""RedisAI in-database inference, MI355X edition (reference `notebooks/redis/RedisAI_TensorFlow.ipynb`
cells 4-30, `data_processing_script_tensorflow.py`): tensors set/get by value and as blobs, a ResNet-50
set as a model on the GPU, TorchScript pre/post-processing set as a script, and the
`SCRIPTRUN pre_process_3ch -> MODELRUN -> SCRIPTRUN post_process` chain timed per image. Tensors stay
in HBM between the three commands.

The TF-Hub resnet_v2_50 frozen graph is downloaded by the notebook; offline the ResNet-50 v2 weights
are random (the predicted index is therefore arbitrary), so the example reports latency. Images:
the reference's JPEGs when $MIFX_REFERENCE_DATA points at a checkout, else synthetic 224x224."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from mifx.models.resnet import resnet50_v2  # noqa: E402
from mifx.models.resnet_infer import FoldedResNetV2  # noqa: E402
from mifx.serving.tensorstore import TensorStore  # noqa: E402

SCRIPT = """
def pre_process_3ch(image):
    return image.float().div(255).unsqueeze(0)

def post_process(output):
    return output.max(1)[1] - 1
"""


def _images() -> dict:
    ref = os.environ.get("MIFX_REFERENCE_DATA", "")
    out = {}
    for name in ("cat", "dog", "guitar", "salvatore"):
        p = os.path.join(ref, "notebooks", "redis", f"{name}.jpg")
        if ref and os.path.exists(p):
            from PIL import Image

            out[name] = np.asarray(Image.open(p).convert("RGB").resize((224, 224)), dtype=np.uint8)
        else:
            out[name] = np.random.default_rng(len(out)).integers(0, 256, (224, 224, 3), dtype=np.uint8)
    return out


def main(repeats: int = 5) -> dict:
    gpu = torch.cuda.is_available()
    dev = "GPU" if gpu else "CPU"
    rai = TensorStore()
    rai.execute_command("AI.TENSORSET", "vector_np", "DOUBLE", 3, "VALUES", 1.0, 2.0, 3.0)
    print("vector_np:", rai.tensorget("vector_np")["values"])
    blob = np.array([1.0, 2.0, 3.0]).tobytes()
    rai.execute_command("AI.TENSORSET", "np_blob", "DOUBLE", 3, "BLOB", blob)
    print("np_blob:", np.frombuffer(rai.tensorget("np_blob", "BLOB"), np.float64))

    torch.manual_seed(0)
    model = resnet50_v2(1001)          # TF-Hub resnet_v2_50 has 1001 classes (0 = background)
    model = model.to(memory_format=torch.channels_last) if gpu else model
    rai.execute_command("AI.MODELSET", "imagenet_model", "TORCH", dev, "INPUTS", "images", "OUTPUTS", "output",
                        _FoldedNHWCModel(model))
    rai.execute_command("AI.SCRIPTSET", "imagenet_script", dev, SCRIPT)

    lat = {}
    for name, img in _images().items():
        times = []
        for _ in range(repeats):
            t0 = time.perf_counter()
            rai.execute_command("AI.TENSORSET", "image", "UINT8", *img.shape, "BLOB", img.tobytes())
            rai.execute_command("AI.SCRIPTRUN", "imagenet_script", "pre_process_3ch", "INPUTS", "image", "OUTPUTS",
                                "temp1")
            rai.execute_command("AI.MODELRUN", "imagenet_model", "INPUTS", "temp1", "OUTPUTS", "temp2")
            rai.execute_command("AI.SCRIPTRUN", "imagenet_script", "post_process", "INPUTS", "temp2", "OUTPUTS", "out")
            pred = rai.execute_command("AI.TENSORGET", "out", "VALUES")
            times.append(time.perf_counter() - t0)
        lat[name] = {"index": int(pred["values"][0]), "first_s": times[0], "steady_s": float(np.median(times[1:]))
                     if len(times) > 1 else times[0]}
        print(f"{name}: predicted index {lat[name]['index']} in {lat[name]['steady_s'] * 1e3:.2f} ms "
              f"(first call {times[0] * 1e3:.1f} ms)")
    print(json.dumps({"device": dev, "latency": lat}))
    return lat


class _FoldedNHWCModel(torch.nn.Module):
    """The served model, taking the [1, H, W, 3] float image the TF-style script produces. On the GPU the eval-mode
    network runs folded (BatchNorms inside the convolutions, mifx.models.resnet_infer) and captured in one hipGraph
    per input shape, built on the first call (after MODELSET moved the module to the device and set eval mode)."""

    def __init__(self, m):
        super().__init__()
        self.m = m
        self._run, self._shape = None, None

    def forward(self, x):
        x = x.permute(0, 3, 1, 2)
        if not x.is_cuda:
            return self.m(x)
        x = x.contiguous(memory_format=torch.channels_last)
        if self._run is None or self._shape != tuple(x.shape):
            self._run, self._shape = FoldedResNetV2(self.m.eval()).graphed(x), tuple(x.shape)
        return self._run(x)


if __name__ == "__main__":
    main()
