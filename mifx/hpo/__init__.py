"""Hyper-parameter search (Katib StudyJob equivalent): random / grid suggestions, parallel trials
pinned one-per-GPU, metrics collected from trial stdout, early stop at the optimisation goal."""
from .study import (GridSuggestion, ParameterConfig, RandomSuggestion, StudyRunner, StudySpec,  # noqa: F401
                    Trial, parse_metrics)
