"""TFX-style pipeline components."""
from .example_gen import CsvExampleGen, ImportExampleGen  # noqa: F401
from .proto import (EvalArgs, FeatureSlicingSpec, Filesystem, PushDestination, SingleSlicingSpec,  # noqa: F401
                    SplitConfig, TrainArgs)
from .statistics import ExampleValidator, SchemaGen, StatisticsGen  # noqa: F401
from .trainer import Evaluator, ModelValidator, Pusher, Trainer  # noqa: F401
from .transform import Transform  # noqa: F401
