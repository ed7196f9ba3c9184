"""Model analysis (TFMA-equivalent): sliced metrics, run_model_analysis, time series."""
from .analysis import (EvalSharedModel, SingleSliceSpec, default_eval_shared_model, load_eval_result,  # noqa: F401
                       load_eval_results, run_model_analysis)
from .metrics import EvalResult, SliceSpec, binary_metrics, compute_sliced_metrics  # noqa: F401
