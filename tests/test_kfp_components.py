"""Components, lightweight Python ops, local workflow execution, local client and CLI.

Reference strategy: `sdk/python/tests/components/test_python_op.py:48-300` (generated program run
as a subprocess with outputs redirected to a temp dir), `test_components.py` (component.yaml
loading, placeholders), `tests/dsl/*` (ops, params). Execution of compiled workflows has no
reference counterpart (the reference relies on an Argo cluster); here it runs on the host."""
import json
import os
import subprocess
import sys
from pathlib import Path
from typing import NamedTuple

import pytest
import yaml

from mifx.kfp import Client, compiler, components, dsl
from mifx.kfp.components._python_op import _func_to_component_spec
from mifx.kfp.local import LocalWorkflowExecutor, evaluate_when
from tests.kfp_testdata.pipelines import PIPELINES


def add_two_numbers(a: float, b: float) -> float:
    """Returns sum of two arguments"""
    return a + b


_SCALE = 10


class _Scaler:
    def scale(self, x):
        return x * _SCALE


def _module_func(a: float) -> float:
    return a * 5


def module_func_with_deps(a: float, b: float) -> float:
    return _Scaler().scale(a) + _module_func(b)


def _run_task(op, *args, tmp_path):
    with components.components_local_output_dir_context(str(tmp_path)):
        task = op(*args)
    subprocess.run(task.command + task.arguments, check=True)
    return task


@pytest.mark.parametrize("func", [add_two_numbers, module_func_with_deps])
def test_func_to_container_op_local_call(func, tmp_path):
    op = components.func_to_container_op(func)
    task = _run_task(op, 3.0, 5.0, tmp_path=tmp_path)
    out = Path(list(task.file_outputs.values())[0]).read_text()
    assert float(out) == func(3.0, 5.0)


def test_named_tuple_outputs(tmp_path):
    def add_multiply(a: float, b: float) -> NamedTuple("Out", [("sum", float), ("product", float)]):
        return (a + b, a * b)

    op = components.func_to_container_op(add_multiply)
    task = _run_task(op, 3.0, 5.0, tmp_path=tmp_path)
    assert float(Path(task.file_outputs["sum"]).read_text()) == 8.0
    assert float(Path(task.file_outputs["product"]).read_text()) == 15.0


def test_same_input_output_names(tmp_path):
    def f(a: float, b: float) -> NamedTuple("Out", [("a", float), ("b", float)]):
        return (a + b, a * b)

    task = _run_task(components.func_to_container_op(f), 3.0, 5.0, tmp_path=tmp_path)
    assert float(Path(task.file_outputs["a"]).read_text()) == 8.0
    assert float(Path(task.file_outputs["b"]).read_text()) == 15.0


def test_bool_inputs_parse_truth_strings(tmp_path):
    def negate(x: bool) -> bool:
        return not x

    task = _run_task(components.func_to_container_op(negate), "False", tmp_path=tmp_path)
    assert Path(list(task.file_outputs.values())[0]).read_text() == "True"


def test_python_component_decorator_and_defaults():
    @dsl.python_component(name="Sum component name", description="Sum component description",
                          base_image="org/image")
    def add_decorated(a: float, b: float = 2.5) -> float:
        return a + b

    spec = _func_to_component_spec(add_decorated)
    assert spec.name == "Sum component name"
    assert spec.description.strip() == "Sum component description"
    assert spec.implementation.container.image == "org/image"
    assert [i.default for i in spec.inputs] == [None, "2.5"]


def test_func_to_component_text_roundtrip(tmp_path):
    text = components.func_to_component_text(add_two_numbers)
    d = yaml.safe_load(text)
    assert d["name"] == "Add two numbers" and d["outputs"] == [{"name": "Output", "type": "float"}]
    op = components.load_component_from_text(text)
    task = _run_task(op, 1.5, 2.0, tmp_path=tmp_path)
    assert float(Path(list(task.file_outputs.values())[0]).read_text()) == 3.5


_COMPONENT = """\
name: Concat
inputs:
- {name: a, type: String}
- {name: b, type: String, default: 'x'}
- {name: flag, type: Bool, optional: true}
outputs:
- {name: joined}
implementation:
  container:
    image: alpine
    command:
    - sh
    - -c
    - {concat: ['echo -n ', {inputValue: a}, {inputValue: b}, ' > ', {outputPath: joined}]}
    args:
    - if:
        cond: {isPresent: flag}
        then: [--flag, {inputValue: flag}]
        else: [--noflag]
"""


def test_load_component_placeholders(tmp_path):
    op = components.load_component_from_text(_COMPONENT)
    with components.components_local_output_dir_context(str(tmp_path)):
        t1 = op("p", "q")
        t2 = op(a="p", flag="true")
    assert t1.arguments == ["--noflag"]
    assert t2.arguments == ["--flag", "true"]
    assert "echo -n pq > " in t1.command[2]
    assert t1.file_outputs["joined"].startswith(str(tmp_path))


def test_component_store(tmp_path):
    d = tmp_path / "lib" / "concat"
    d.mkdir(parents=True)
    (d / "component.yaml").write_text(_COMPONENT)
    store = components.ComponentStore(local_search_paths=[str(tmp_path / "lib")])
    op = store.load_component("concat")
    assert op.component_spec.name == "Concat"
    with pytest.raises(RuntimeError):
        store.load_component("missing")


def test_evaluate_when():
    assert evaluate_when("heads == heads") and not evaluate_when("heads == tails")
    assert evaluate_when("10 > 9") and evaluate_when("1.5 <= 1.5") and evaluate_when("a != b")
    assert evaluate_when("1 == 1 && 2 == 2") and not evaluate_when("1 == 2 && 2 == 2")


def _run_local(pipeline, tmp_path, args=None):
    wf = compiler.Compiler().compile_to_workflow(pipeline)
    return LocalWorkflowExecutor(wf, str(tmp_path / "run"), args, max_parallel=4).run()


def test_local_executor_coin_conditions(tmp_path):
    st = _run_local(PIPELINES["coin"], tmp_path)
    assert st["phase"] == "Succeeded", st["message"]
    nodes = {n["name"]: n for n in st["nodes"].values()}
    flip = next(n for k, n in nodes.items() if k.endswith(".flip"))
    res = flip["outputs"]["parameters"][0]["value"]
    assert res in ("heads", "tails")
    ran = {k.rsplit(".", 1)[-1] for k, n in nodes.items() if n["phase"] == "Succeeded"}
    assert ("condition-1" in ran) == (res == "heads")
    assert ("condition-3" in ran) == (res == "tails")


def test_local_executor_recursion_terminates(tmp_path):
    st = _run_local(PIPELINES["recursive_while"], tmp_path)
    assert st["phase"] == "Succeeded", st["message"]
    # the closing print (after the loop) always runs; the in-loop print runs once per "heads"
    assert any(n["templateName"].startswith("print") for n in st["nodes"].values() if n["phase"] == "Succeeded")


def test_local_executor_retry_and_exit_handler(tmp_path):
    marker = tmp_path / "attempts"

    @dsl.pipeline(name="retry exit")
    def p():
        exit_op = dsl.ContainerOp(name="cleanup", image="alpine", command=["sh", "-c"],
                                  arguments=[f"echo {{{{workflow.status}}}} > {tmp_path}/exit_status"])
        with dsl.ExitHandler(exit_op):
            dsl.ContainerOp(name="flaky", image="alpine", command=["sh", "-c"],
                            arguments=[f"echo x >> {marker}; test $(wc -l < {marker}) -ge 3"]).set_retry(5)

    st = _run_local(p, tmp_path)
    assert st["phase"] == "Succeeded", st["message"]
    assert len(marker.read_text().splitlines()) == 3
    assert (tmp_path / "exit_status").read_text().strip() == "Succeeded"


def test_local_executor_failure_propagates(tmp_path):
    @dsl.pipeline(name="fails")
    def p():
        a = dsl.ContainerOp(name="bad", image="alpine", command=["sh", "-c", "exit 3"])
        dsl.ContainerOp(name="after", image="alpine", command=["true"]).after(a)

    st = _run_local(p, tmp_path)
    assert st["phase"] == "Failed" and "exit code 3" in st["message"]
    assert not any(n["name"].endswith(".after") for n in st["nodes"].values())


def test_local_executor_python_components_dataflow(tmp_path):
    add = components.func_to_container_op(add_two_numbers)

    @dsl.pipeline(name="adder")
    def p(a: float = 1.0, b: float = 2.0):
        s = add(a, b)
        add(s.output, 10.0)

    st = _run_local(p, tmp_path, {"a": "4"})
    assert st["phase"] == "Succeeded", st["message"]
    vals = sorted(float(n["outputs"]["parameters"][0]["value"]) for n in st["nodes"].values()
                  if n["templateName"].startswith("add-two-numbers"))
    assert vals == [6.0, 16.0]


def test_client_local_backend(tmp_path):
    add = components.func_to_container_op(add_two_numbers)

    @dsl.pipeline(name="client adder")
    def p(a: float = 1.0, b: float = 2.0):
        add(a, b)

    pkg = str(tmp_path / "p.tar.gz")
    compiler.Compiler().compile(p, pkg)
    client = Client(host=f"local://{tmp_path / 'store'}")
    exp = client.create_experiment("exp1")
    assert client.create_experiment("exp1").id == exp.id  # idempotent by name
    run = client.run_pipeline(exp.id, "job", pkg, {"a": 5})
    detail = client.wait_for_run_completion(run.id, timeout=120)
    assert detail.run.status == "Succeeded"
    wf = client._get_workflow_json(run.id)
    assert wf["status"]["phase"] == "Succeeded"
    runs = client.list_runs(experiment_id=exp.id)
    assert [r.id for r in runs.runs] == [run.id]
    pl = client.upload_pipeline(pkg, "adder")
    run2 = client.run_pipeline(exp.id, "job2", pipeline_id=pl.id)
    assert client.wait_for_run_completion(run2.id, timeout=120).run.status == "Succeeded"


def test_cli_run_list_and_submit(tmp_path):
    pkg = str(tmp_path / "p.yaml")
    compiler.Compiler().compile(PIPELINES["retry"], pkg)
    env_store = f"local://{tmp_path / 'store'}"
    r = subprocess.run([sys.executable, "-m", "mifx.kfp", "--endpoint", env_store, "run", "submit", "-e", "e1",
                        "-f", pkg, "-w"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "is submitted" in r.stdout and "finished with status" in r.stdout
    r = subprocess.run([sys.executable, "-m", "mifx.kfp", "--endpoint", env_store, "run", "list"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "e1" in r.stdout


def test_compat_aliases():
    from mifx.kfp import compat

    compat.install()
    import kfp  # noqa: F401
    import kfp.dsl as kdsl
    from kubernetes import client as k8s_client

    assert kdsl.ContainerOp is dsl.ContainerOp
    assert k8s_client.V1EnvVar(name="a", value="b").to_dict() == {"name": "a", "value": "b"}


def test_amd_gpu_modifier():
    from mifx.kfp import amd

    @dsl.pipeline(name="gpu")
    def p():
        dsl.ContainerOp(name="train", image="rocm/pytorch", command=["python3", "train.py"]).apply(
            amd.use_amd_gpus(8)).apply(amd.use_torchrun(8))

    wf = compiler.Compiler()._compile(p)
    t = next(t for t in wf["spec"]["templates"] if t["name"] == "train")
    assert t["container"]["resources"]["limits"]["amd.com/gpu"] == "8"
    assert t["nodeSelector"]["amd.com/gpu.product-name"] == "MI355X"
    assert {"name": "HSA_ENABLE_IPC_MODE_LEGACY", "value": "0"} in t["container"]["env"]
    assert t["container"]["command"][:3] == ["python3", "-m", "torch.distributed.run"]
    assert any(v["name"] == "dshm" for v in wf["spec"]["volumes"])


def test_component_builder_artifacts(tmp_path):
    from mifx.kfp.compiler._component_builder import (DependencyHelper, DockerfileHelper, ImageBuilder,
                                                      VersionedDependency)

    h = DependencyHelper()
    h.add_python_package(VersionedDependency("tensorflow", min_version="0.10.0", max_version="0.11.0"))
    h.add_python_package(VersionedDependency("kubernetes", min_version="0.6.0"))
    h.add_python_package(VersionedDependency("pytorch", max_version="0.3.0"))
    req = tmp_path / "req.txt"
    h.generate_pip_requirements(str(req))
    assert req.read_text() == ("tensorflow >= 0.10.0, <= 0.11.0\nkubernetes >= 0.6.0\npytorch <= 0.3.0\n"
                               .replace(", <=", ", <="))
    df = DockerfileHelper("dockerfile").dockerfile_text("gcr.io/ngunwu/tensorflow", "main.py", True)
    assert df.splitlines()[0] == "FROM gcr.io/ngunwu/tensorflow"
    assert df.splitlines()[-1] == 'ENTRYPOINT ["python3", "/ml/main.py"]'
    assert "RUN pip3 install -r /ml/requirements.txt" in df

    def sample(a: int, b: str) -> str:
        return b * a

    code = ImageBuilder(str(tmp_path / "stage"), "img")._generate_entrypoint(sample)
    prog = tmp_path / "main.py"
    prog.write_text(code)
    out = tmp_path / "o" / "data"
    subprocess.run([sys.executable, str(prog), "3", "ab", str(out)], check=True)
    assert out.read_text() == "ababab"


def test_workflow_status_written(tmp_path):
    st = _run_local(PIPELINES["retry"], tmp_path)
    with open(tmp_path / "run" / "status.json") as f:
        assert json.load(f)["phase"] == st["phase"]


def test_pipelines_api_server_with_rest_client(tmp_path):
    import threading

    import uvicorn

    from mifx.kfp.server import create_app
    from tests.test_parallel_cpu import _free_port

    port = _free_port()
    server = uvicorn.Server(uvicorn.Config(create_app(str(tmp_path / "api")), host="127.0.0.1", port=port,
                                           log_level="error"))
    th = threading.Thread(target=server.run, daemon=True)
    th.start()
    try:
        import time as _t

        for _ in range(100):
            if server.started:
                break
            _t.sleep(0.05)
        pkg = str(tmp_path / "p.tar.gz")
        compiler.Compiler().compile(PIPELINES["retry"], pkg)
        client = Client(host=f"http://127.0.0.1:{port}", poll_interval=0.2)
        exp = client.create_experiment("rest-exp")
        assert client.get_experiment(experiment_name="rest-exp").id == exp.id
        run = client.run_pipeline(exp.id, "rest-run", pkg, {})
        detail = client.wait_for_run_completion(run.id, timeout=120)
        assert detail.run.status in ("Succeeded", "Failed")  # random failures are the sample's point
        assert client.list_runs(experiment_id=exp.id).runs[0].id == run.id
        pl = client.upload_pipeline(pkg, "retry")
        assert any(p.id == pl.id for p in client.list_pipelines().pipelines)
        # the pipelines UI on the same port: index, the run's graph (an SVG box per executed node), the pipeline DAG
        import requests

        idx = requests.get(f"http://127.0.0.1:{port}/", timeout=10)
        assert idx.status_code == 200 and "rest-run" in idx.text and f"/ui/runs/{run.id}" in idx.text
        page = requests.get(f"http://127.0.0.1:{port}/ui/runs/{run.id}", timeout=10).text
        wf = client._get_workflow_json(run.id)
        assert "<svg" in page and page.count("<rect") >= 1 and detail.run.status in page
        assert page.count("<rect") == len(wf["status"]["nodes"])
        pp = requests.get(f"http://127.0.0.1:{port}/ui/pipelines/{pl.id}", timeout=10)
        assert pp.status_code == 200 and "<table>" in pp.text
        assert requests.get(f"http://127.0.0.1:{port}/ui/runs/nope", timeout=10).status_code == 404
    finally:
        server.should_exit = True
        th.join(timeout=10)


def test_pipelines_ui_layout_and_escaping():
    from mifx.kfp import ui

    pos = ui.layout({"a": ["b", "c"], "b": ["d"], "c": ["d"], "d": []})
    assert pos["a"][0] == 0 and pos["b"][0] == pos["c"][0] == 1 and pos["d"][0] == 2
    assert ui._e("<script>") == "&lt;script&gt;"


def test_local_executor_deep_recursion_keeps_step_dirs_short(tmp_path):
    """A graph component recursing 12 levels: the nested display path outgrows the file-name limit,
    so step sandboxes are named by a bounded prefix/digest/suffix (executor._exec_container)."""
    from mifx.kfp import compiler, dsl
    from mifx.kfp.local import LocalWorkflowExecutor

    def dec_op(n):
        return dsl.ContainerOp(name="decrement-counter-step", image="python:3.10-alpine", command=["sh", "-c"],
                               arguments=['python3 -c "import sys; print(int(sys.argv[1]) - 1)" $0 | tee $1', n,
                                          "/tmp/output"], file_outputs={"output": "/tmp/output"})

    @dsl.graph_component
    def count_down(n):
        nxt = dec_op(n)
        with dsl.Condition(nxt.output > 0):
            count_down(nxt.output)

    @dsl.pipeline(name="deep recursion")
    def deep(start=12):
        count_down(start)

    wf = compiler.Compiler().compile_to_workflow(deep)
    st = LocalWorkflowExecutor(wf, str(tmp_path), {"start": "12"}, timeout=300).run()
    assert st["phase"] == "Succeeded", st
    steps = os.listdir(tmp_path / "steps")
    assert len([s for s in steps if "decrement" in s]) == 12
    assert max(len(s) for s in steps) <= 120
