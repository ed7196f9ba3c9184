"""Differential privacy: RDP accountant, private queries, DP optimizers (fused HIP clip/noise), PATE."""
from . import pate, queries, rdp  # noqa: F401
from .optimizers import (DPAdagradOptimizer, DPAdamOptimizer, DPGradientDescentOptimizer,  # noqa: F401
                         DPOptimizer, make_optimizer_class, sparse_softmax_ce)
from .rdp import compute_dp_sgd_privacy, compute_rdp, get_privacy_spent  # noqa: F401
