"""KFP taxi preprocessing module for the `tft` step (same transforms as the reference's
`kubeflow-pipelines/taxi/preprocessing.py:26-102`): z-score the 3 dense floats, vocabulary
(top 1000 + 10 OOV) for 6 features (ints stringified first), 10 quantile buckets for lat/lon,
hour/day/month passed through, label = !isnan(fare) && tips > 0.2 * fare. No `_xf` suffix."""
import numpy as np

import mifx.transform as mt
from mifx.models.taxi_dnn import (BUCKET_FEATURE_KEYS, CATEGORICAL_FEATURE_KEYS, DENSE_FLOAT_FEATURE_KEYS,
                                  FEATURE_BUCKET_COUNT, LABEL_KEY, OOV_SIZE, VOCAB_FEATURE_KEYS, VOCAB_SIZE)

FARE_KEY = "fare"


def _floats(x):
    return np.array([np.nan if v is None else float(v) for v in np.asarray(x, dtype=object)], dtype=np.float64)


def preprocess(inputs):
    out = {}
    for key in DENSE_FLOAT_FEATURE_KEYS:
        v = _floats(inputs[key])
        v = np.where(np.isnan(v), np.nanmean(v) if np.isfinite(v).any() else 0.0, v)  # nan -> mean
        out[key] = mt.scale_to_z_score(v)
    for key in VOCAB_FEATURE_KEYS:
        out[key] = mt.string_to_int(mt.as_string(mt.fill_in_missing(inputs[key])), top_k=VOCAB_SIZE,
                                    num_oov_buckets=OOV_SIZE, vocab_filename="vocab_" + key)
    for key in BUCKET_FEATURE_KEYS:
        out[key] = mt.bucketize(mt.fill_in_missing(_floats(inputs[key])), FEATURE_BUCKET_COUNT)
    for key in CATEGORICAL_FEATURE_KEYS:
        out[key] = np.nan_to_num(_floats(inputs[key])).astype(np.int64)
    fare, tips = _floats(inputs[FARE_KEY]), _floats(inputs[LABEL_KEY])
    out[LABEL_KEY] = np.logical_and(~np.isnan(fare), tips > fare * 0.2).astype(np.int64)
    return out
