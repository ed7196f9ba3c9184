"""TFDV-equivalent statistics/schema/anomalies and tf.Transform-equivalent analyzers."""
import numpy as np
import pandas as pd
import pytest

import mifx.data_validation as dv
import mifx.transform as mt
from mifx.io import tfrecord


def _df(seed=0, n=500, shift=0.0):
    r = np.random.default_rng(seed)
    return pd.DataFrame({"fare": r.gamma(2, 5, n) + shift, "company": r.choice(["a", "b", "c"], n, p=[.6, .3, .1]),
                         "hour": r.integers(0, 24, n), "tips": r.gamma(1, 1, n)})


def test_stats_schema_pbtxt_roundtrip():
    st = dv.generate_statistics_from_dataframe(_df())
    f = dv.get_feature_stats(st, "fare")
    assert f["num_stats"]["common_stats"]["num_non_missing"] == 500
    assert abs(f["num_stats"]["mean"] - _df()["fare"].mean()) < 1e-9
    schema = dv.infer_schema(st)
    assert schema.get_feature("company").domain == "company"
    assert schema.get_domain("company").value == ["a", "b", "c"]
    text = schema.to_pbtxt()
    back = dv.Schema.from_pbtxt(text)
    assert back.to_pbtxt() == text
    assert "fare" in dv.stats_frame(st).index


def test_anomalies_domain_mass_environment_and_skew():
    train = dv.generate_statistics_from_dataframe(_df())
    schema = dv.infer_schema(train)
    ev = _df(1)
    ev.loc[:20, "company"] = "zzz"
    evs = dv.generate_statistics_from_dataframe(ev)
    an = dv.validate_statistics(evs, schema)
    assert "company" in an.anomaly_info
    assert an.anomaly_info["company"]["reason"][0]["type"] == "ENUM_TYPE_UNEXPECTED_STRING_VALUES"
    schema.get_feature("company").min_domain_mass = 0.9  # relax (notebook cell 19)
    assert not dv.validate_statistics(evs, schema)
    serving = dv.generate_statistics_from_dataframe(_df(2).drop(columns=["tips"]))
    assert "tips" in dv.validate_statistics(serving, schema).anomaly_info
    schema.default_environment = ["TRAINING", "SERVING"]
    schema.get_feature("tips").not_in_environment = ["SERVING"]
    assert not dv.validate_statistics(serving, schema, environment="SERVING")
    schema.get_feature("company").skew_linf_threshold = 0.01
    skewed = _df(3)
    skewed["company"] = "a"
    an = dv.validate_statistics(train, schema, serving_statistics=dv.generate_statistics_from_dataframe(skewed))
    assert an.anomaly_info["company"]["reason"][0]["type"] == "COMPARATOR_L_INFTY_HIGH"


def _pf(inputs):
    x = inputs["x"]
    return {"x_z": mt.scale_to_z_score(x), "x_01": mt.scale_to_0_1(x), "x_mean_sub": x - mt.mean(x),
            "s_id": mt.compute_and_apply_vocabulary(inputs["s"], top_k=2, num_oov_buckets=3),
            "x_b": mt.bucketize(x, 4)}


def test_transform_analyze_then_apply_replays_constants():
    # notebook 03 toy example semantics
    inputs = {"x": np.array([1.0, 2.0, 3.0, 4.0]), "s": np.array(["hello", "world", "hello", "hello"], object)}
    out, st = mt.analyze(_pf, inputs)
    assert np.allclose(out["x_z"], (inputs["x"] - 2.5) / inputs["x"].std())
    assert np.allclose(out["x_01"], [0, 1 / 3, 2 / 3, 1])
    assert out["s_id"].tolist() == [0, 1, 0, 0]  # frequency-desc vocabulary
    assert sorted(set(out["x_b"].tolist())) == [0, 1, 2, 3]
    new = {"x": np.array([2.5]), "s": np.array(["unseen"], object)}
    res = mt.apply(_pf, new, mt.TransformState.from_json(st.to_json()))
    assert res["x_mean_sub"][0] == pytest.approx(0.0)
    assert 2 <= res["s_id"][0] < 5  # OOV bucket after the 2-entry vocab


def test_vocab_ties_break_by_value_descending():
    out, st = mt.analyze(lambda i: {"v": mt.compute_and_apply_vocabulary(i["s"])},
                         {"s": np.array(["b", "a", "c", "c"], object)})
    assert st.entries[0]["values"] == ["c", "b", "a"]


def test_fill_in_missing():
    assert mt.fill_in_missing(np.array([None, "x"], object)).tolist() == ["", "x"]
    assert mt.fill_in_missing(np.array([1.0, np.nan])).tolist() == [1.0, 0.0]
    assert mt.fill_in_missing(np.array([None, 3], object)).tolist() == [0, 3]
    # ints mixed with strings stay a string column (pandas infers "mixed-integer"): no value is coerced to NaN
    assert mt.fill_in_missing(np.array([None, 3, "a"], object)).tolist() == ["", 3, "a"]
    assert mt.fill_in_missing(np.array([1.5, None, "b"], object)).tolist() == [1.5, "", "b"]


def test_tfrecord_roundtrip_and_corruption(tmp_path):
    assert tfrecord.crc32c(b"123456789") == 0xE3069283
    recs = [tfrecord.encode_example({"a": [i, -i], "f": np.array([0.5], np.float32), "s": [b"x" * i]})
            for i in range(5)]
    p = str(tmp_path / "r.tfrecord")
    tfrecord.write_tfrecords(p, recs, "")
    back = [tfrecord.decode_example(r) for r in tfrecord.read_tfrecords(p)]
    assert back[3] == {"a": [3, -3], "f": [0.5], "s": [b"xxx"]}
    raw = bytearray(open(p, "rb").read())
    raw[20] ^= 0xFF
    open(p, "wb").write(bytes(raw))
    with pytest.raises(IOError):
        list(tfrecord.read_tfrecords(p))
