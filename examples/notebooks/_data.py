"""Data for the notebook-equivalent examples: the reference's Chicago-taxi CSVs when a checkout is
mounted at $MIFX_REFERENCE_DATA (read as plain CSV text), otherwise synthetic rows with the same 18
columns (`mifx.data.synthetic.synthetic_taxi_csv_rows`)."""
from __future__ import annotations

import os
import sys

import pandas as pd

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.data.synthetic import synthetic_taxi_csv_rows  # noqa: E402

_REF = os.environ.get("MIFX_REFERENCE_DATA", "")


def taxi_csvs(workdir: str, n_train: int = 10000, n_eval: int = 5000, seed: int = 0) -> tuple[str, str]:
    """(train.csv, eval.csv) paths: reference `kubeflow-pipelines/taxi/{train,eval}.csv` if available."""
    if _REF:
        tr = os.path.join(_REF, "kubeflow-pipelines", "taxi", "train.csv")
        ev = os.path.join(_REF, "kubeflow-pipelines", "taxi", "eval.csv")
        if os.path.exists(tr) and os.path.exists(ev):
            return tr, ev
    os.makedirs(workdir, exist_ok=True)
    tr, ev = os.path.join(workdir, "train.csv"), os.path.join(workdir, "eval.csv")
    pd.DataFrame(synthetic_taxi_csv_rows(n_train, seed=seed)).to_csv(tr, index=False)
    eval_df = pd.DataFrame(synthetic_taxi_csv_rows(n_eval, seed=seed + 1))
    # the eval split of the reference carries a few unseen categorical values (notebook 02, cell 17)
    if "company" in eval_df and len(eval_df) > 10:
        eval_df.loc[eval_df.index[:max(1, len(eval_df) // 100)], "company"] = "Unseen Cab Co"
        eval_df.loc[eval_df.index[:max(1, len(eval_df) // 200)], "payment_type"] = "Mobile"
    eval_df.to_csv(ev, index=False)
    return tr, ev
