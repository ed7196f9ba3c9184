"""PATE: teacher ensembles, noisy aggregation, and privacy analysis (2017 moments, 2018 RDP)."""
from . import aggregation, analysis2017, rdp2018, smooth_sensitivity  # noqa: F401
