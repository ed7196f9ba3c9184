"""tf.Transform-equivalent preprocessing: analyzers (full pass) + mappers (per row).

Usage in a user module (cf. `airflow-dags/taxi_utils.py:106-145`)::

    import mifx.transform as mt
    def preprocessing_fn(inputs):
        return {"fare_xf": mt.scale_to_z_score(mt.fill_in_missing(inputs["fare"])), ...}
"""
from .api import (TransformState, analyze, apply, apply_buckets, apply_vocabulary, as_string, bucketize,  # noqa: F401
                  compute_and_apply_vocabulary, fill_in_missing, fingerprint64, hash_strings, max, mean, min,
                  quantiles, scale_by_min_max, scale_to_0_1, scale_to_z_score, size, state_summary, string_to_int,
                  sum, to_float, var, vocabulary)
from .output import TransformOutput, import_module_file, write_transform_output  # noqa: F401
