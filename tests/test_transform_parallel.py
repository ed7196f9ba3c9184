"""Sharded (Beam-style) analyze + transform (mifx.transform.parallel) against the one-process analyze: the same
analyzer state (vocabularies, quantile boundaries and sizes exactly; moments to fp64 rounding) and the same
transformed rows in the same order. Real worker processes (spawned) on the CPU."""
import os

import numpy as np
import pytest

import mifx.transform as mt
from mifx.transform import parallel as tpar


def _data(n, seed=0):
    rng = np.random.default_rng(seed)
    fare = rng.gamma(2.0, 7.0, n)
    fare[rng.random(n) < 0.02] = np.nan
    miles = np.round(rng.exponential(3.0, n), 2)  # many ties
    hour = rng.integers(0, 24, n)
    company = np.array([None if rng.random() < 0.05 else f"co{int(v)}" for v in rng.zipf(1.6, n) % 300],
                       dtype=object)
    return {"fare": fare, "miles": miles, "hour": hour, "company": company}


def preprocessing_fn(inputs):
    fare = mt.fill_in_missing(inputs["fare"])
    out = {
        "fare_xf": mt.scale_to_z_score(fare),
        "miles_b": mt.bucketize(inputs["miles"], 10),
        "hour_01": mt.scale_to_0_1(inputs["hour"]),
        "company_xf": mt.compute_and_apply_vocabulary(mt.fill_in_missing(inputs["company"]), top_k=50,
                                                      num_oov_buckets=3),
        "n": np.full(len(inputs["hour"]), mt.size(inputs["hour"])),
    }
    # an analyzer over a column that depends on an earlier analyzer's merged value
    out["fare_xf_b"] = mt.bucketize(out["fare_xf"], 4)
    out["fare_sum"] = np.full(len(fare), mt.sum(fare))
    return out


def _first_quantiles(st):
    return next(e for e in st.entries if e["kind"] == "quantiles")


@pytest.mark.parametrize("workers", [2, 3])
def test_sharded_analyze_matches_one_process(workers):
    d = _data(20011)
    cols1, st1 = mt.analyze(preprocessing_fn, d)
    cols2, st2 = tpar.analyze_sharded(preprocessing_fn, d, num_workers=workers)
    assert [e["kind"] for e in st1.entries] == [e["kind"] for e in st2.entries]
    for e1, e2 in zip(st1.entries, st2.entries):
        if e1["kind"] == "moments":
            for k in ("mean", "var", "min", "max", "count"):
                np.testing.assert_allclose(e2["values"][k], e1["values"][k], rtol=1e-12)
        elif e1["kind"] == "sum":
            np.testing.assert_allclose(e2["values"], e1["values"], rtol=1e-12)
        else:  # vocabulary, quantiles (exact order statistics), size
            if e1["kind"] == "quantiles" and e1 is not _first_quantiles(st1):
                # over the z-scored fare: its input carries the merged moments' fp64 rounding
                assert len(e1["values"]) == len(e2["values"])
                np.testing.assert_allclose(e2["values"], e1["values"], rtol=1e-12)
                continue
            assert e1["values"] == e2["values"], e1["kind"]
    assert set(cols1) == set(cols2)
    for k in cols1:
        a, b = np.asarray(cols1[k]), np.asarray(cols2[k])
        assert a.shape == b.shape
        if a.dtype.kind == "f":
            np.testing.assert_allclose(b, a, rtol=1e-9, atol=1e-12)
        else:
            assert np.array_equal(a, b), k


def test_sharded_quantiles_exact_on_heavy_ties_and_small_gather(monkeypatch):
    """Force several narrowing rounds (tiny GATHER / bin count) on a column with a dominant repeated value."""
    monkeypatch.setattr(tpar, "GATHER", 8)
    monkeypatch.setattr(tpar, "SELECT_BINS", 16)
    rng = np.random.default_rng(3)
    x = np.concatenate([np.full(5000, 2.5), rng.normal(0, 1, 3000), rng.normal(10, 0.001, 1000)])
    rng.shuffle(x)

    def fn(inputs):
        return {"q": mt.bucketize(inputs["x"], 20)}

    _, st1 = mt.analyze(fn, {"x": x})
    # the workers are spawned: they see the module defaults, so patch through an env-free path -- run in-process
    inits = [tpar._q_init(part) for part in np.array_split(x, 3)]

    class _Local:  # the driver's worker protocol, in-process over three shards
        def __init__(self, parts):
            self.parts = parts

        def call(self, msg):
            op, _, iv = msg
            f = tpar._q_hist if op == "qhist" else tpar._q_gather
            return [f(p, iv) for p in self.parts]

    n = sum(i["n"] for i in inits)
    qs = tpar._distributed_order_stats(_Local(np.array_split(x, 3)), 0, inits, tpar._ranks_higher(n, 20))
    assert sorted(set(float(v) for v in qs)) == st1.entries[0]["values"]


def test_transform_component_num_workers(tmp_path):
    """The Transform component with num_workers=2 writes the same transformed examples as in-process."""
    import csv

    from mifx.components import CsvExampleGen, SchemaGen, StatisticsGen, Transform
    from mifx.orchestration.artifact import csv_input
    from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows
    from mifx.io import dataset
    from mifx.orchestration import LocalDagRunner
    from mifx.orchestration.pipeline import Pipeline

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    module = os.path.join(root, "examples", "taxi", "taxi_module.py")
    data = tmp_path / "data"
    data.mkdir()
    with open(data / "data.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
        w.writeheader()
        for r in synthetic_taxi_csv_rows(3000, seed=2):
            w.writerow({k: ("" if v is None else v) for k, v in r.items()})
    outs = []
    for nw in (0, 2):
        eg = CsvExampleGen(input_base=csv_input(str(data)))
        sg = StatisticsGen(input_data=eg.outputs.examples)
        sc = SchemaGen(stats=sg.outputs.output)
        tf = Transform(input_data=eg.outputs.examples, schema=sc.outputs.output, module_file=module, num_workers=nw)
        p = Pipeline(pipeline_name=f"tp{nw}", pipeline_root=str(tmp_path / f"r{nw}"), components=[eg, sg, sc, tf],
                     metadata_db_root=str(tmp_path / f"md{nw}"))
        assert LocalDagRunner(device="cpu").run(p).succeeded
        arts = {a.split: a for a in tf.outputs.transformed_examples.get()}
        outs.append({s: dataset.read_split(a.uri).to_pandas() for s, a in arts.items()})
    assert set(outs[0]) == set(outs[1]) == {"train", "eval"}
    for split in outs[0]:
        a, b = outs[0][split], outs[1][split]
        assert list(a.columns) == list(b.columns) and len(a) == len(b)
        for c in a.columns:
            if a[c].dtype.kind == "f":
                np.testing.assert_allclose(b[c].to_numpy(), a[c].to_numpy(), rtol=1e-9, atol=1e-12)
            else:
                assert (a[c].to_numpy() == b[c].to_numpy()).all(), c


def test_sharded_quantiles_with_infinities_terminate_and_match():
    """A column with +-inf: the sharded selection bins the finite range only and resolves the infinite tails
    directly (before, linspace over [-inf, hi] made every edge NaN and a crowded bin never narrowed)."""
    rng = np.random.default_rng(5)
    x = np.concatenate([rng.normal(0, 1, 4000), [np.inf] * 300, [-np.inf] * 700])
    rng.shuffle(x)
    parts = np.array_split(x, 3)
    inits = [tpar._q_init(p) for p in parts]

    class _Local:
        def call(self, msg):
            op, _, iv = msg
            f = tpar._q_hist if op == "qhist" else tpar._q_gather
            return [f(p, iv) for p in parts]

    n = sum(i["n"] for i in inits)
    ranks = tpar._ranks_higher(n, 20)
    qs = tpar._distributed_order_stats(_Local(), 0, inits, ranks)
    assert np.array_equal(qs, np.sort(x)[ranks])
    assert qs[0] == -np.inf and qs[-1] == np.inf
