"""Transform component: analyze the train split with the user's `preprocessing_fn`, persist the
transform graph, and materialise transformed examples for every split.

Reference: `Transform(input_data=..., schema=..., module_file=...)` -> outputs `transform_output`
(TransformPath) and `transformed_examples` (ExamplesPath) (`airflow-dags/taxi_pipeline.py:86-89`).
"""
from __future__ import annotations

import os

import numpy as np
import pyarrow as pa

from .. import data_validation as dv
from .. import transform as mt
from ..io import dataset
from ..orchestration import artifact as A
from ..orchestration.component import BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec, ExecutionParameter
from .statistics import load_schema_from_artifact


def table_to_inputs(table: pa.Table, arrow_strings: bool = False) -> dict:
    """Arrow columns -> numpy (object arrays with None for missing strings/ints, NaN floats).
    `arrow_strings`: string columns stay Arrow arrays (offsets + bytes buffers) so the GPU vocabulary
    kernels consume them without a per-row Python pass (mifx.transform.api accepts both forms)."""
    out = {}
    for name in table.column_names:
        col = table.column(name)
        if arrow_strings and (pa.types.is_string(col.type) or pa.types.is_large_string(col.type)):
            out[name] = col
        elif pa.types.is_floating(col.type):
            out[name] = col.to_numpy(zero_copy_only=False).astype(np.float64)
        elif col.null_count or pa.types.is_string(col.type) or pa.types.is_large_string(col.type):
            out[name] = np.array(col.to_pylist(), dtype=object)
        else:
            out[name] = col.to_numpy(zero_copy_only=False)
    return out


def outputs_to_table(cols: dict) -> pa.Table:
    arrs = {}
    for k, v in cols.items():
        v = np.asarray(v)
        if v.dtype == object:
            arrs[k] = pa.array(v.tolist())
        elif v.dtype == bool:
            arrs[k] = pa.array(v.astype(np.int64))
        else:
            arrs[k] = pa.array(v)
    return pa.table(arrs)


class TransformSpec(ComponentSpec):
    PARAMETERS = {"module_file": ExecutionParameter(), "preprocessing_fn_name": ExecutionParameter(
        optional=True, default="preprocessing_fn"), "num_workers": ExecutionParameter(optional=True, default=0)}
    INPUTS = {"input_data": ChannelParameter(A.EXAMPLES), "schema": ChannelParameter(A.SCHEMA)}
    OUTPUTS = {"transform_output": ChannelParameter(A.TRANSFORM),
               "transformed_examples": ChannelParameter(A.EXAMPLES)}


class TransformExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        module_file = exec_properties["module_file"]
        fn_name = exec_properties.get("preprocessing_fn_name") or "preprocessing_fn"
        fn = mt.import_module_file(module_file, fn_name)
        splits = {a.split: a for a in input_dict["input_data"]}
        train = splits.get("train") or next(iter(splits.values()))
        raw_schema = load_schema_from_artifact(input_dict["schema"][0].uri)
        dev = self.context.device
        gpu = dev is not None and str(dev).startswith("cuda")
        table = dataset.read_split(train.uri)
        workers = int(exec_properties.get("num_workers") or 0)
        if workers > 1:  # Beam-style: shards on worker processes, merged accumulators (mifx.transform.parallel)
            from ..transform import parallel as tpar

            cols, state = tpar.analyze_sharded(fn, table_to_inputs(table), num_workers=workers)
        else:
            cols, state = self._analyze_local(fn, table, dev, gpu)
        t_stats = dv.generate_statistics_from_table(outputs_to_table(cols), name="train")
        t_schema = dv.infer_schema(t_stats)
        out = output_dict["transform_output"][0]
        mt.write_transform_output(out.uri, state, module_file, fn_name, t_schema.to_pbtxt(), raw_schema.to_pbtxt())
        for art in output_dict["transformed_examples"]:
            if art.split == train.split:
                res = cols
            elif workers > 1:
                res = tpar.transform_sharded(fn, table_to_inputs(dataset.read_split(splits[art.split].uri)), state,
                                             num_workers=workers)
            else:
                res = mt.apply(fn, table_to_inputs(dataset.read_split(splits[art.split].uri)), state, device=dev)
            dataset.write_split(art.uri, outputs_to_table(res))
            art.custom_properties["num_examples"] = int(len(next(iter(res.values()))))

    @staticmethod
    def _analyze_local(fn, table, dev, gpu):
        try:
            cols, state = mt.analyze(fn, table_to_inputs(table, arrow_strings=gpu), device=dev)
        except (TypeError, AttributeError, ValueError):
            if not gpu:
                raise
            # user code that needs numpy string columns: same analysis on the numpy form
            cols, state = mt.analyze(fn, table_to_inputs(table), device=dev)
        return cols, state


class Transform(BaseComponent):
    SPEC_CLASS = TransformSpec
    EXECUTOR_CLASS = TransformExecutor
    EXECUTION_TYPE = "transform"

    def __init__(self, input_data, schema, module_file: str, preprocessing_fn_name: str = "preprocessing_fn",
                 name: str | None = None, transform_output=None, transformed_examples=None, num_workers: int = 0):
        """num_workers > 1: analyze + transform sharded over that many worker processes (the reference's Beam
        DirectRunner with `--direct_num_workers`; mifx.transform.parallel)."""
        super().__init__(TransformSpec(input_data=input_data, schema=schema, module_file=os.path.abspath(module_file),
                                       preprocessing_fn_name=preprocessing_fn_name, num_workers=int(num_workers),
                                       transform_output=transform_output,
                                       transformed_examples=transformed_examples), name=name)

    def output_splits(self, key, input_dict):
        if key == "transformed_examples":
            return [a.split for a in input_dict["input_data"]]
        return [""]
