"""Notebook 09_Advanced_KubeFlow_ML_Pipeline (reference: upload the compiled taxi pipeline package in the
Pipelines UI and start a run from it). Here: compile the KFP taxi pipeline (`examples/kfp/taxi`), upload
the package to the pipelines backend (`Client.upload_pipeline`), list it with its parameters, and --
with `--run` -- start a run from the uploaded pipeline id, as the UI's "Create run" does."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "kfp", "taxi")))

import mifx.kfp as kfp  # noqa: E402
import mifx.kfp.compiler as compiler  # noqa: E402
from taxi_pipeline import taxi_cab_classification  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="local")
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "mifx_n09"))
    ap.add_argument("--run", action="store_true", help="start a run from the uploaded pipeline")
    a = ap.parse_args(argv)
    os.makedirs(a.workdir, exist_ok=True)
    package = os.path.join(a.workdir, "taxi-cab-classification-pipeline.tar.gz")
    compiler.Compiler().compile(taxi_cab_classification, package)
    host = a.host if a.host != "local" else f"local://{os.path.join(a.workdir, 'kfp')}"
    client = kfp.Client(host=host)
    pipeline = client.upload_pipeline(package, "taxi-cab-classification-pipeline")
    listed = client.list_pipelines(page_size=50).pipelines
    print("uploaded:", pipeline.id, [p["name"] for p in listed])
    print("parameters:", [p["name"] for p in pipeline.parameters])
    out = {"pipeline": pipeline, "listed": listed, "run": None}
    if a.run:
        exp = client.create_experiment("taxi")
        out["run"] = client.run_pipeline(exp.id, "taxi run", pipeline_id=pipeline.id)
        print("run:", out["run"].id)
    return out


if __name__ == "__main__":
    main()
