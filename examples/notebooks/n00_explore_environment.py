"""Notebook 00_Explore_Environment (reference `notebooks/00_Explore_Environment.ipynb` cell 4: framework and
Python versions, accelerator discovery) for the MI355X stack: Python / PyTorch / ROCm (HIP) versions, the
visible GPUs with their gfx arch, CU count and HBM size, RCCL availability, and whether this package's
gfx950 HIP libraries are built (`mifx.utils.env.report`)."""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.utils import env  # noqa: E402


def main() -> dict:
    rep = env.report()
    print(json.dumps(rep, indent=2, default=str))
    return rep


if __name__ == "__main__":
    main()
