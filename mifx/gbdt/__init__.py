"""Gradient-boosted trees with the XGBRegressor/XGBClassifier API used by the fairing XGBoost sample
(`kubeflow-pipelines/fairing/fairing_xgboost.py:60-87`: n_estimators=1000, learning_rate=0.1,
early_stopping_rounds=50 on an eval_set, best_score/best_iteration). CPU plug-in (out of
GPU scope); the histogram GBDT core is scikit-learn's, driven round by round so early stopping on the
caller's eval set (RMSE / logloss) matches XGBoost's semantics."""
from .xgb import XGBClassifier, XGBRegressor  # noqa: F401
