"""The KFP DSL feature tour of `kubeflow-pipelines/basic/*.py` (README `basic/README.md:1-30`) as one
module of runnable mifx pipelines: sequential steps, a parallel fan-in, nested conditions, an exit
handler, recursion through a graph component, per-op retries, a pipeline-wide op transformer, a
sidecar, an immediate-value parameter and a pipeline-level artifact location.

The reference steps download from GCS with `gsutil`; here the "download" step reads a local file
through the same shape of container op (`sh -c 'cat $0 | tee $1'`), so every sample except the
sidecar (it needs a pod network) compiles AND runs on this host through the local Argo-equivalent
executor:

    python examples/kfp/basic_samples.py --compile-only out_dir     # Argo packages (.zip)
    python examples/kfp/basic_samples.py --run sequential           # run one locally
"""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.kfp import compiler, dsl  # noqa: E402
from mifx.kfp.k8s import V1SecretKeySelector  # noqa: E402

PY = "python3"  # runs on the host with the local executor; in-cluster use a python image
IMG_PY = "python:3.10-alpine"
IMG_SH = "bash:5"


def read_op(path, out="/tmp/results.txt"):
    """'Download' a text: cat the file and keep it as the step output `data`."""
    return dsl.ContainerOp(name="download", image=IMG_SH, command=["sh", "-c"],
                           arguments=["cat $0 | tee $1", path, out], file_outputs={"data": out})


def echo_op(*texts):
    script = "; ".join(f'echo "Text {i + 1}: ${i}"' for i in range(len(texts))) if len(texts) > 1 else 'echo "$0"'
    return dsl.ContainerOp(name="echo", image=IMG_SH, command=["sh", "-c"], arguments=[script, *texts])


def coin_op():
    return dsl.ContainerOp(name="flip-coin", image=IMG_PY, command=["sh", "-c"],
                           arguments=[f"{PY} -c \"import random; print('heads' if random.randint(0, 1) == 0 "
                                      "else 'tails')\" | tee /tmp/output"],
                           file_outputs={"output": "/tmp/output"})


def random_num_op(low, high):
    return dsl.ContainerOp(name="random-number", image=IMG_PY, command=["sh", "-c"],
                           arguments=[f'{PY} -c "import random; print(random.randint($0, $1))" | tee $2',
                                      str(low), str(high), "/tmp/output"],
                           file_outputs={"output": "/tmp/output"})


def print_op(msg):
    return dsl.ContainerOp(name="print", image="alpine:3", command=["echo", msg])


def failing_op(exit_codes):
    """Exits with a random code from the list (the reference's fault-injection op)."""
    return dsl.ContainerOp(name="random-failure", image=IMG_PY, command=[PY, "-c"],
                           arguments=["import random, sys; c = int(random.choice(sys.argv[1].split(','))); "
                                      "print(c); sys.exit(c)", exit_codes])


# ---------------------------------------------------------------------------------- samples
@dsl.pipeline(name="Sequential pipeline", description="Two sequential steps.")
def sequential(url="/etc/hostname"):
    echo_op(read_op(url).output)


@dsl.pipeline(name="Parallel pipeline", description="Two reads in parallel, joined by one step.")
def parallel_join(url1="/etc/hostname", url2="/etc/os-release"):
    echo_op(read_op(url1).output, read_op(url2).output)


@dsl.pipeline(name="Conditional execution pipeline", description="Nested dsl.Condition blocks.")
def condition():
    flip = coin_op()
    for side, lo, hi, mid in (("heads", 0, 9, 5), ("tails", 10, 19, 15)):
        with dsl.Condition(flip.output == side):
            n = random_num_op(lo, hi)
            with dsl.Condition(n.output > mid):
                print_op(f"{side} and {n.output} > {mid}!")
            with dsl.Condition(n.output <= mid):
                print_op(f"{side} and {n.output} <= {mid}!")


@dsl.pipeline(name="Exit Handler", description="The exit step runs whether the body succeeds or not.")
def exit_handler(url="/etc/hostname"):
    done = echo_op("exit!")
    with dsl.ExitHandler(done):
        echo_op(read_op(url).output)


@dsl.graph_component
def flip_until_tails(flip_result):
    shown = print_op(flip_result)
    again = coin_op().after(shown)
    with dsl.Condition(again.output == "heads"):
        flip_until_tails(again.output)


@dsl.pipeline(name="Recursive loop pipeline", description="Recursion through a graph component.")
def recursion():
    loop = flip_until_tails(coin_op().output)
    print_op("cool, it is over.").after(loop)


@dsl.pipeline(name="Retry random failures", description="Per-op set_retry.")
def retry():
    failing_op("0,1,2,3").set_retry(10)
    failing_op("0,1").set_retry(5)


@dsl.pipeline(name="Retry via op transformer", description="add_op_transformer applies a retry to every op.")
def pipeline_transformers():
    failing_op("0,1,2,3")
    failing_op("0,1")

    def add_retry(op):
        op.set_retry(5)
        return op

    dsl.get_pipeline_conf().add_op_transformer(add_retry)


@dsl.pipeline(name="pipeline_with_sidecar", description="An op with an HTTP echo sidecar.")
def sidecar(sleep_ms: int = 10):
    echo = dsl.Sidecar(name="echo", image="hashicorp/http-echo:latest", args=['-text="hello world"'])
    op1 = dsl.ContainerOp(name="download", image="busybox:latest", command=["sh", "-c"],
                          arguments=[f"sleep {sleep_ms}; wget localhost:5678 -O /tmp/results.txt"],
                          sidecars=[echo], file_outputs={"downloaded": "/tmp/results.txt"})
    dsl.ContainerOp(name="echo", image="bash:5", command=["sh", "-c"], arguments=[f"echo {op1.output}"])


@dsl.pipeline(name="Immediate Value", description="A parameter whose value is fixed in the pipeline.")
def immediate_value():
    url = dsl.PipelineParam(name="url", value="/etc/hostname")
    op1 = dsl.ContainerOp(name="download", image=IMG_SH, command=["sh", "-c"],
                          arguments=[f"cat {url} | tee /tmp/results.txt"],
                          file_outputs={"downloaded": "/tmp/results.txt"})
    dsl.ContainerOp(name="echo", image=IMG_SH, command=["sh", "-c"], arguments=[f"echo {op1.output}"])


@dsl.pipeline(name="custom_artifact_location_pipeline", description="Pipeline-level S3/Minio artifact location.")
def artifact_location(tag: str = "latest", namespace: str = "kubeflow", bucket: str = "mybucket"):
    loc = dsl.ArtifactLocation.s3(bucket=bucket, endpoint=f"minio-service.{namespace}:9000", insecure=True,
                                  access_key_secret=V1SecretKeySelector(name="minio", key="accesskey"),
                                  secret_key_secret={"name": "minio", "key": "secretkey"})
    dsl.get_pipeline_conf().set_artifact_location(loc)
    dsl.ContainerOp(name="foo", image=f"busybox:{tag}", command=["sh", "-c"], arguments=["echo stored"])


SAMPLES = {f.__name__: f for f in (sequential, parallel_join, condition, exit_handler, recursion, retry,
                                   pipeline_transformers, sidecar, immediate_value, artifact_location)}
LOCAL_RUNNABLE = [k for k in SAMPLES if k != "sidecar"]


def compile_all(out_dir: str) -> dict:
    os.makedirs(out_dir, exist_ok=True)
    out = {}
    for name, fn in SAMPLES.items():
        out[name] = os.path.join(out_dir, name + ".zip")
        compiler.Compiler().compile(fn, out[name])
    return out


def run_local(name: str, run_dir: str, arguments: dict | None = None) -> dict:
    from mifx.kfp.local import LocalWorkflowExecutor

    wf = compiler.Compiler().compile_to_workflow(SAMPLES[name])
    return LocalWorkflowExecutor(wf, run_dir, arguments, timeout=300).run()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--compile-only", metavar="OUT_DIR")
    ap.add_argument("--run", choices=sorted(SAMPLES), nargs="*")
    a = ap.parse_args(argv)
    if a.compile_only:
        for k, v in compile_all(a.compile_only).items():
            print(f"{k:>22} -> {v}")
    for name in a.run or []:
        st = run_local(name, os.path.join(tempfile.gettempdir(), "mifx_kfp_basic", name))
        print(f"{name:>22}: {st['phase']}")


if __name__ == "__main__":
    main()
