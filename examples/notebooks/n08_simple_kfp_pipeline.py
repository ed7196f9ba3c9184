"""Notebook 08 (simple Kubeflow pipeline) with mifx.kfp (reference
`notebooks/08_Simple_KubeFlow_ML_Pipeline.ipynb` cells 3-17): lightweight components from Python
functions (single output `add_fn`, NamedTuple multi-output `div_fn` that also writes
mlpipeline-metrics.json), compile to an Argo package, create an experiment and submit a run.

With `--host local` (default) the run executes on this machine through the local Argo-equivalent
executor; pass the URL of a `mifx-pipelines-api` server to submit over REST instead."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile
from typing import NamedTuple

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import mifx.kfp as kfp  # noqa: E402
import mifx.kfp.compiler as compiler  # noqa: E402
import mifx.kfp.components as comp  # noqa: E402
import mifx.kfp.dsl as dsl  # noqa: E402


def add_fn(a: float, b: float) -> float:
    '''Calculates sum of two arguments'''
    return a + b


def div_fn(dividend: float, divisor: float, output_dir: str = './') -> NamedTuple('DivOutput', [('quotient', float), ('remainder', float)]):  # noqa: E501,F821
    '''Divides two numbers and calculate  the quotient and remainder'''
    import numpy as np

    def nested_div_helper(dividend, divisor):
        return np.divmod(dividend, divisor)

    (quotient, remainder) = nested_div_helper(dividend, divisor)

    import json
    metrics = {'metrics': [{'name': 'quotient', 'numberValue': float(quotient)},
                           {'name': 'remainder', 'numberValue': float(remainder)}]}
    with open(output_dir + 'mlpipeline-metrics.json', 'w') as f:
        json.dump(metrics, f)

    from collections import namedtuple
    output = namedtuple('DivOutput', ['quotient', 'remainder'])
    return output(quotient, remainder)


add_op = comp.func_to_container_op(add_fn)
div_op = comp.func_to_container_op(div_fn, base_image='rocm/pytorch:latest')


@dsl.pipeline(name='Calculation pipeline', description='A toy pipeline that performs arithmetic calculations.')
def add_div_pipeline(a='a', b='7', c='17'):
    add_task = add_op(a, 4)
    # in-cluster the notebook passes '/', the container root; the local executor runs each step in
    # its own sandbox directory, so the metrics file goes to the step's working directory
    div_task = div_op(add_task.output, b, './')
    add_op(div_task.outputs['quotient'], c)


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default="local")
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "mifx_n08"))
    a = ap.parse_args(argv)
    os.makedirs(a.workdir, exist_ok=True)
    print("div_fn(100, 7) =", div_fn(100, 7, a.workdir + os.sep))
    pipeline_filename = os.path.join(a.workdir, add_div_pipeline.__name__ + '.pipeline.tar.gz')
    compiler.Compiler().compile(add_div_pipeline, pipeline_filename)
    arguments = {'a': '7', 'b': '8'}
    host = a.host if a.host != "local" else f"local://{os.path.join(a.workdir, 'kfp')}"
    client = kfp.Client(host=host)
    experiment = client.create_experiment('simple_add_div_pipeline')
    run_result = client.run_pipeline(experiment.id, add_div_pipeline.__name__ + ' run', pipeline_filename, arguments)
    done = client.wait_for_run_completion(run_result.id, timeout=300)
    print("run", run_result.id, "->", done.run.status if hasattr(done, "run") else done)
    return {"run": done, "package": pipeline_filename}


if __name__ == "__main__":
    main()
