"""Run the 9-component Chicago-Taxi pipeline (reference config: 15,000 rows, Trainer 10,000 train / 5,000 eval
steps at batch 40, checkpoints every 999 steps -- airflow-dags/taxi_pipeline.py:97-98, taxi_utils.py:333-334)
under LocalDagRunner on one device and write per-component times, the Trainer's examples/sec and the eval
metrics as one JSON object.

    python tools/pipeline_bench.py --device cuda --out profiles/archive/pipeline_gpu_r3.json
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples", "taxi"))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--rows", type=int, default=15000)
    ap.add_argument("--train-steps", type=int, default=10000)
    ap.add_argument("--eval-steps", type=int, default=5000)
    ap.add_argument("--batch-size", type=int, default=40)
    ap.add_argument("--num-gpus", type=int, default=1)
    ap.add_argument("--gpu-min-rows", type=int, default=None,
                    help="run the Transform analyzers on the GPU from this column size (default: the library's)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)

    import taxi_pipeline_local as tp

    import mifx.transform.api as tapi
    from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows
    from mifx.orchestration import LocalDagRunner

    if a.gpu_min_rows is not None:
        tapi.GPU_MIN_ROWS = a.gpu_min_rows
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "data"))
        with open(os.path.join(d, "data", "data.csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
            w.writeheader()
            for r in synthetic_taxi_csv_rows(a.rows, seed=1):
                w.writerow({k: ("" if v is None else v) for k, v in r.items()})
        p = tp.create_pipeline("taxi", os.path.join(d, "root"), os.path.join(d, "data"), os.path.join(d, "serving"),
                               train_steps=a.train_steps, eval_steps=a.eval_steps,
                               metadata_db_root=os.path.join(d, "md"), batch_size=a.batch_size,
                               num_gpus=a.num_gpus)
        t0 = time.time()
        res = LocalDagRunner(device=a.device).run(p)
        wall = time.time() - t0
        tr = res.components["Trainer"].outputs["output"][0]
        m = json.load(open(os.path.join(tr.uri, "metrics.json")))
        ckpts = sorted(os.listdir(os.path.join(tr.uri, "serving_model_dir")))
        out = {"device": a.device, "rows": a.rows, "train_steps": a.train_steps, "eval_steps": a.eval_steps,
               "batch_per_replica": a.batch_size, "num_gpus": a.num_gpus, "succeeded": res.succeeded,
               "pipeline_wall_s": wall,
               "component_seconds": {k: round(c.seconds, 3) for k, c in res.components.items()},
               "trainer_examples_per_sec": m.get("train_examples_per_sec"), "trainer_global_step": m.get("global_step"),
               "checkpoints_left": [c for c in ckpts if c.startswith("ckpt-")],
               "eval": m.get("eval"), "gpu_min_rows": tapi.GPU_MIN_ROWS,
               "data": "synthetic Chicago-Taxi-shaped CSV (no network for the real data)"}
    line = json.dumps(out, default=float)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")
    return 0 if out["succeeded"] else 1


if __name__ == "__main__":
    raise SystemExit(main())
