"""Notebook 03 (TensorFlow Transform basics) with mifx.transform
(reference `notebooks/03_TensorFlow_Transform.ipynb` cells 7-9): three toy rows through
mean / scale_to_0_1 / compute_and_apply_vocabulary in one analyze-and-transform pass."""
from __future__ import annotations

import os
import pprint
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402

import mifx.transform as tft  # noqa: E402

raw_data = [
    {"x": 1, "y": 1, "s": "hello"},
    {"x": 2, "y": 2, "s": "world"},
    {"x": 3, "y": 3, "s": "hello"},
]


def preprocessing_fn(inputs):
    x, y, s = inputs["x"], inputs["y"], inputs["s"]
    x_centered = x - tft.mean(x)
    y_normalized = tft.scale_to_0_1(y)
    s_integerized = tft.compute_and_apply_vocabulary(s)
    return {
        "x_centered": x_centered,
        "y_normalized": y_normalized,
        "s_integerized": s_integerized,
        "x_centered_times_y_normalized": x_centered * y_normalized,
    }


def main() -> list[dict]:
    cols = {k: np.array([r[k] for r in raw_data], dtype=object if k == "s" else np.float32) for k in raw_data[0]}
    out, _state = tft.analyze(preprocessing_fn, cols)
    transformed = [{k: (v[i].item() if hasattr(v[i], "item") else v[i]) for k, v in out.items()}
                   for i in range(len(raw_data))]
    print("\nRaw data:\n{}\n".format(pprint.pformat(raw_data)))
    print("Transformed data:\n{}".format(pprint.pformat(transformed)))
    return transformed


if __name__ == "__main__":
    main()
