"""StatisticsGen / SchemaGen / ExampleValidator components.

Reference: `StatisticsGen(input_data=...)`, `SchemaGen(stats=...)`,
`ExampleValidator(stats=..., schema=...)` (`airflow-dags/taxi_pipeline.py:76-83`); artifacts
hold `stats.json` per split (TFDV stats), `schema.pbtxt` (`06_Airflow_Feature_Analysis.ipynb:L76`)
and `anomalies.json`.
"""
from __future__ import annotations

import os

from .. import data_validation as dv
from ..data_validation.stats import load_statistics, stats_frame  # noqa: F401  (re-export for lineage)
from ..io import dataset
from ..orchestration import artifact as A
from ..orchestration.component import BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec, ExecutionParameter


def _by_split(arts):
    return {a.split: a for a in arts}


# --------------------------------------------------------------------------- StatisticsGen
class StatisticsGenSpec(ComponentSpec):
    INPUTS = {"input_data": ChannelParameter(A.EXAMPLES)}
    OUTPUTS = {"output": ChannelParameter(A.EXAMPLE_STATS)}


class StatisticsGenExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        ins = _by_split(input_dict["input_data"])
        for art in output_dict["output"]:
            table = dataset.read_split(ins[art.split].uri)
            st = dv.generate_statistics_from_table(table, name=art.split, device=self.context.device)
            dv.write_stats(st, os.path.join(art.uri, "stats.json"))


class StatisticsGen(BaseComponent):
    SPEC_CLASS = StatisticsGenSpec
    EXECUTOR_CLASS = StatisticsGenExecutor
    EXECUTION_TYPE = "statistics_gen"

    def __init__(self, input_data, name: str | None = None, output=None):
        super().__init__(StatisticsGenSpec(input_data=input_data, output=output), name=name)

    def output_splits(self, key, input_dict):
        return [a.split for a in input_dict["input_data"]]


# ------------------------------------------------------------------------------- SchemaGen
class SchemaGenSpec(ComponentSpec):
    PARAMETERS = {"infer_feature_shape": ExecutionParameter(optional=True, default=True)}
    INPUTS = {"stats": ChannelParameter(A.EXAMPLE_STATS)}
    OUTPUTS = {"output": ChannelParameter(A.SCHEMA)}


class SchemaGenExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        stats = _by_split(input_dict["stats"])
        src = stats.get("train") or next(iter(stats.values()))
        schema = dv.infer_schema(load_statistics(src.uri), bool(exec_properties.get("infer_feature_shape", True)))
        dv.write_schema_text(schema, os.path.join(output_dict["output"][0].uri, "schema.pbtxt"))


class SchemaGen(BaseComponent):
    SPEC_CLASS = SchemaGenSpec
    EXECUTOR_CLASS = SchemaGenExecutor
    EXECUTION_TYPE = "schema_gen"

    def __init__(self, stats, infer_feature_shape: bool = True, name: str | None = None, output=None):
        super().__init__(SchemaGenSpec(stats=stats, infer_feature_shape=infer_feature_shape, output=output), name=name)


def load_schema_from_artifact(uri: str) -> dv.Schema:
    return dv.load_schema_text(os.path.join(uri, "schema.pbtxt"))


# ------------------------------------------------------------------------ ExampleValidator
class ExampleValidatorSpec(ComponentSpec):
    INPUTS = {"stats": ChannelParameter(A.EXAMPLE_STATS), "schema": ChannelParameter(A.SCHEMA)}
    OUTPUTS = {"output": ChannelParameter(A.EXAMPLE_VALIDATION)}


class ExampleValidatorExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        schema = load_schema_from_artifact(input_dict["schema"][0].uri)
        out = output_dict["output"][0]
        total = 0
        for st in input_dict["stats"]:
            env = None
            an = dv.validate_statistics(load_statistics(st.uri), schema, environment=env)
            total += len(an.anomaly_info)
            with open(os.path.join(out.uri, f"anomalies_{st.split or 'all'}.json"), "w") as f:
                f.write(an.to_json())
        out.custom_properties["num_anomalies"] = total


class ExampleValidator(BaseComponent):
    SPEC_CLASS = ExampleValidatorSpec
    EXECUTOR_CLASS = ExampleValidatorExecutor
    EXECUTION_TYPE = "example_validation"

    def __init__(self, stats, schema, name: str | None = None, output=None):
        super().__init__(ExampleValidatorSpec(stats=stats, schema=schema, output=output), name=name)
