"""Columnar split storage for example artifacts.

An Examples artifact URI holds ``data-SSSSS-of-NNNNN.parquet`` shards (Arrow columnar: typed,
null-aware, mmap-able) and, optionally, gzip TFRecords of tf.Example for TF tooling
compatibility (`airflow-dags/taxi_utils.py:79-83`).
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from . import tfrecord


def to_table(data) -> pa.Table:
    if isinstance(data, pa.Table):
        return data
    if isinstance(data, dict):
        return pa.table({k: pa.array(v) for k, v in data.items()})
    import pandas as pd

    if isinstance(data, pd.DataFrame):
        return pa.Table.from_pandas(data, preserve_index=False)
    raise TypeError(f"cannot convert {type(data).__name__} to an Arrow table")


def write_split(uri: str, data, num_shards: int = 1, tfrecords: bool = False) -> list[str]:
    os.makedirs(uri, exist_ok=True)
    table = to_table(data)
    n = table.num_rows
    paths = []
    for s in range(num_shards):
        lo, hi = n * s // num_shards, n * (s + 1) // num_shards
        p = os.path.join(uri, f"data-{s:05d}-of-{num_shards:05d}.parquet")
        pq.write_table(table.slice(lo, hi - lo), p)
        paths.append(p)
    if tfrecords:
        write_tfrecord_split(uri, table)
    return paths


def read_split(uri: str, columns: list[str] | None = None) -> pa.Table:
    files = sorted(glob.glob(os.path.join(uri, "data-*.parquet")))
    if not files:
        tfr = sorted(glob.glob(os.path.join(uri, "*.gz")) + glob.glob(os.path.join(uri, "*.tfrecord")))
        if tfr:
            return read_tfrecord_split(uri)
        raise FileNotFoundError(f"no example shards under {uri}")
    t = pa.concat_tables([pq.read_table(f, columns=columns) for f in files])
    return t


def table_to_numpy(table: pa.Table) -> dict[str, np.ndarray]:
    out = {}
    for name in table.column_names:
        col = table.column(name)
        if pa.types.is_string(col.type) or pa.types.is_large_string(col.type):
            out[name] = np.array(col.to_pylist(), dtype=object)
        elif pa.types.is_integer(col.type):
            if col.null_count:
                out[name] = np.array(col.to_pylist(), dtype=object)
            else:
                out[name] = col.to_numpy().astype(np.int64)
        else:
            out[name] = col.to_numpy(zero_copy_only=False).astype(np.float64)
    return out


def write_tfrecord_split(uri: str, table: pa.Table, name: str = "data_tfrecord-00000-of-00001.gz") -> str:
    rows = table.to_pylist()

    def gen():
        for r in rows:
            feats = {}
            for k, v in r.items():
                if v is None:
                    feats[k] = []  # missing -> empty list (sparse column of rank <= 1)
                elif isinstance(v, str):
                    feats[k] = [v.encode()]
                elif isinstance(v, float):
                    feats[k] = np.asarray([v], np.float32)
                else:
                    feats[k] = [int(v)]
            yield tfrecord.encode_example(feats)

    p = os.path.join(uri, name)
    tfrecord.write_tfrecords(p, gen(), "GZIP")
    return p


def read_tfrecord_split(uri: str) -> pa.Table:
    rows = []
    for f in sorted(glob.glob(os.path.join(uri, "*.gz")) + glob.glob(os.path.join(uri, "*.tfrecord"))):
        for rec in tfrecord.read_tfrecords(f):
            ex = tfrecord.decode_example(rec)
            rows.append({k: (None if not v else (v[0].decode() if isinstance(v[0], bytes) else v[0]))
                         for k, v in ex.items()})
    return pa.Table.from_pylist(rows)
