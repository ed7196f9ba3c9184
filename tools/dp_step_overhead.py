"""Host/GPU cost of the data-parallel W&D step paths on ONE GPU with a 1-rank RCCL group: the split-phase
step (graph, eager RCCL all-reduce, graph), the direct path bench.py uses at N>1 (eager kernel launches from
prebuilt arguments + ncclAllReduce on the same stream), and the single graph with the all-reduce captured
(include_collective=True), and the xGMI one-shot exchange (its 1-rank exchange still publishes/waits on the
epoch flag and reads the partial back; whole step in 10-step graphs). The trainer is told world=2 so it takes
the DP code path."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mifx.data.synthetic import synthetic_records  # noqa: E402
from mifx.models.wide_deep import WideDeepModel  # noqa: E402
from mifx.trainer.fused_wide_deep import FusedWideDeepTrainer  # noqa: E402


def run(batch, include_collective, steps=300, dp_mode="split"):
    tr = FusedWideDeepTrainer(WideDeepModel(seed=0), batch=batch, device="cuda", process_group=dist.group.WORLD)
    tr.world = 2  # force the DP path (reduce_full -> all_reduce -> optimizer) on a 1-rank group
    tr.set_data(synthetic_records(1 << 20, device="cuda", seed=1))
    tr.capture(include_collective=include_collective, dp_mode=dp_mode,
               steps_per_graph=10 if dp_mode == "xgmi" else 1)
    tr.run(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(steps)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    return {"batch": batch, "captured_collective": include_collective, "dp_mode": dp_mode,
            "host_us_per_step": round(t_host / steps * 1e6, 2),
            "us_per_step": round(t_all / steps * 1e6, 2), "finite": bool(torch.isfinite(tr.param).all()),
            "xgmi_err": int(tr._xg.err.item()) if tr._xg is not None else None}


if __name__ == "__main__":
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
    torch.cuda.set_device(0)
    if len(sys.argv) > 1:  # e.g. `xgmi` (one mode, B=65536; for kernel traces)
        print(json.dumps(run(65536, False, dp_mode=sys.argv[1])), flush=True)
        dist.destroy_process_group()
        sys.exit(0)
    for b in (65536, 40):
        print(json.dumps(run(b, False, dp_mode="split")), flush=True)
    for b in (65536, 40):
        print(json.dumps(run(b, False, dp_mode="direct")), flush=True)
    for b in (65536, 40):
        print(json.dumps(run(b, True)), flush=True)
    for b in (65536, 40):
        print(json.dumps(run(b, False, dp_mode="xgmi")), flush=True)
    dist.destroy_process_group()
