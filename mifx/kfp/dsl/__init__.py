"""KFP-v0.1-compatible pipeline DSL (reference: `sdk/python/kfp/dsl/__init__.py`)."""
from ._artifact_location import ArtifactLocation  # noqa: F401
from ._component import component, graph_component, python_component  # noqa: F401
from ._container_op import BaseOp, Container, ContainerOp, Sidecar  # noqa: F401
from ._metadata import ComponentMeta, ParameterMeta, PipelineMeta, TypeMeta  # noqa: F401
from ._ops_group import Condition, ExitHandler, Graph, OpsGroup  # noqa: F401
from ._pipeline import Pipeline, PipelineConf, get_pipeline_conf, pipeline  # noqa: F401
from ._pipeline_param import (ConditionOperator, PipelineParam, extract_pipelineparams_from_any,  # noqa: F401
                              match_serialized_pipelineparam, sanitize_k8s_name)
from ._pipeline_volume import PipelineVolume  # noqa: F401
from ._resource_op import (VOLUME_MODE_ROM, VOLUME_MODE_RWM, VOLUME_MODE_RWO, Resource, ResourceOp,  # noqa: F401
                           VolumeOp, VolumeSnapshotOp)
