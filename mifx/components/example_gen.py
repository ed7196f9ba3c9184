"""ExampleGen: ingest CSV (or Parquet / TFRecord) into hash-split example artifacts.

Reference: `CsvExampleGen(input_base=csv_input(data_root))` (`airflow-dags/taxi_pipeline.py:70-73`),
TFX 0.13 semantics: deterministic hash split of every record into train:eval = 2:1, outputs one
ExamplesPath artifact per split, later read by StatisticsGen/Transform/Evaluator/ModelValidator.
Records are stored as Parquet shards (+ optional gzip tf.Example TFRecords, `output_tfrecords`).
"""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.parquet as pq

from ..io import dataset
from ..orchestration import artifact as A
from ..orchestration.component import (BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec,
                                       ExecutionParameter)
from .proto import SplitConfig, default_splits


def _read_input(uri: str) -> pa.Table:
    files = [uri] if os.path.isfile(uri) else sorted(os.path.join(uri, f) for f in os.listdir(uri))
    tables = []
    for f in files:
        if f.endswith(".csv"):
            tables.append(pacsv.read_csv(f))
        elif f.endswith(".parquet"):
            tables.append(pq.read_table(f))
        elif f.endswith((".gz", ".tfrecord")):
            tables.append(dataset.read_tfrecord_split(os.path.dirname(f)))
    if not tables:
        raise FileNotFoundError(f"no .csv/.parquet/.tfrecord input under {uri}")
    return pa.concat_tables(tables, promote_options="default")


def hash_split(table: pa.Table, splits: list[SplitConfig]) -> dict[str, pa.Table]:
    """Deterministic per-record split by hashing the serialized row (TFX ExampleGen partition)."""
    n = table.num_rows
    total = sum(s.hash_buckets for s in splits)
    cols = [table.column(c).to_pylist() for c in table.column_names]
    bucket = np.empty(n, dtype=np.int64)
    for i in range(n):
        key = "\x1f".join("" if c[i] is None else repr(c[i]) for c in cols).encode()
        bucket[i] = int.from_bytes(hashlib.md5(key).digest()[:8], "little") % total
    out, lo = {}, 0
    for s in splits:
        idx = np.nonzero((bucket >= lo) & (bucket < lo + s.hash_buckets))[0]
        out[s.name] = table.take(pa.array(idx))
        lo += s.hash_buckets
    return out


class ExampleGenSpec(ComponentSpec):
    PARAMETERS = {"input_config": ExecutionParameter(optional=True), "output_config": ExecutionParameter(optional=True),
                  "output_tfrecords": ExecutionParameter(optional=True, default=False),
                  "num_shards": ExecutionParameter(optional=True, default=1)}
    INPUTS = {"input_base": ChannelParameter(A.EXTERNAL)}
    OUTPUTS = {"examples": ChannelParameter(A.EXAMPLES)}


class ExampleGenExecutor(BaseExecutor):
    def Do(self, input_dict, output_dict, exec_properties):  # noqa: N802
        table = _read_input(input_dict["input_base"][0].uri)
        splits = [SplitConfig(**s) if isinstance(s, dict) else s
                  for s in (exec_properties.get("output_config") or default_splits())]
        parts = hash_split(table, splits)
        for art in output_dict["examples"]:
            t = parts[art.split]
            dataset.write_split(art.uri, t, num_shards=int(exec_properties.get("num_shards") or 1),
                                tfrecords=bool(exec_properties.get("output_tfrecords")))
            art.custom_properties["num_examples"] = t.num_rows
        self.context.logger.info("ExampleGen: %s", {k: v.num_rows for k, v in parts.items()})


class CsvExampleGen(BaseComponent):
    SPEC_CLASS = ExampleGenSpec
    EXECUTOR_CLASS = ExampleGenExecutor
    EXECUTION_TYPE = "examples_gen"

    def __init__(self, input_base, output_config: list | None = None, output_tfrecords: bool = False,
                 num_shards: int = 1, name: str | None = None, examples=None):
        splits = [s.to_dict() if isinstance(s, SplitConfig) else s for s in (output_config or default_splits())]
        super().__init__(ExampleGenSpec(input_base=input_base, output_config=splits, output_tfrecords=output_tfrecords,
                                        num_shards=num_shards, examples=examples), name=name)
        self._split_names = [s["name"] for s in splits]

    def output_splits(self, key, input_dict):
        return list(self._split_names)


ImportExampleGen = CsvExampleGen  # accepts parquet / tfrecord inputs as well
