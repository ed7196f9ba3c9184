"""Utilities: TensorBoard-compatible summaries, throughput meter, trace ranges."""
from .meter import ExamplesPerSec, trace_range  # noqa: F401
from .summary import SummaryWriter, read_scalars  # noqa: F401
