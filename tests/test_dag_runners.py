"""KubeflowDagRunner (compile -> execute each component in its own process via the local Argo
executor, artifacts handed over through MLMD) and AirflowDagRunner (DAG source / local fallback)."""
import json
import os

from mifx.kfp.local import LocalWorkflowExecutor
from mifx.metadata.store import MetadataStore
from mifx.orchestration import AirflowDagRunner, KubeflowDagRunner, KubeflowDagRunnerConfig
from tests.kfp_testdata.tfx_factory import create_pipeline

ROOT = os.path.dirname(os.path.dirname(__file__))
FACTORY = "tests.kfp_testdata.tfx_factory:create_pipeline"


def test_kubeflow_dag_runner_executes_per_component(tmp_path):
    args = {"root": str(tmp_path / "p")}
    p = create_pipeline(**args)
    runner = KubeflowDagRunner(KubeflowDagRunnerConfig(pvc_name=None, gpu_components={"StatisticsGen": 1}))
    wf = runner.compile(p, FACTORY, args)
    t = {x["name"]: x for x in wf["spec"]["templates"]}
    assert {"csvexamplegen", "statisticsgen", "schemagen"} <= set(t)
    assert t["statisticsgen"]["container"]["resources"]["limits"]["amd.com/gpu"] == "1"
    env = dict(os.environ, PYTHONPATH=ROOT)
    st = LocalWorkflowExecutor(wf, str(tmp_path / "run"), env=env).run()
    assert st["phase"] == "Succeeded", st["message"]
    store = MetadataStore(p.metadata_connection_config)
    names = sorted({e.properties["component_id"].string_value for e in store.get_executions()})
    assert names == ["CsvExampleGen", "SchemaGen", "StatisticsGen"]
    # lineage: SchemaGen's input is StatisticsGen's output in the same run
    schema_ex = [e for e in store.get_executions() if e.properties["component_id"].string_value == "SchemaGen"][0]
    ins = [e for e in store.get_events_by_execution_ids([schema_ex.id]) if e.type == 1 or e.type == 3]
    assert ins
    store.close()


def test_airflow_dag_runner_source_and_local_fallback(tmp_path):
    args = {"root": str(tmp_path / "p")}
    p = create_pipeline(**args)
    r = AirflowDagRunner({"schedule_interval": None, "start_date": (2019, 1, 1)})
    src = r.dag_source(p, FACTORY, args)
    compile(src, "dag.py", "exec")
    assert src.count("BashOperator(") == 3 and "tasks['CsvExampleGen'] >> tasks['StatisticsGen']" in src
    assert json.loads(json.loads(src.split("--factory-args '\" + ")[1].split(" + \"'")[0]))["root"] == args["root"]
    res = r.run(p)  # airflow not installed -> in-process run
    assert res.succeeded
