"""Op model: Container / Sidecar (k8s container wrappers), BaseOp, ContainerOp.

Reference: `sdk/python/kfp/dsl/_container_op.py:96-1083`. `set_gpu_limit(gpu, vendor)` accepts
'nvidia' or 'amd' and emits `<vendor>.com/gpu`; on this framework 'amd' is the natural choice
(see :mod:`mifx.kfp.amd` for MI355X node selectors and ROCm device plumbing).
"""
from __future__ import annotations

import re
import warnings
from typing import Callable

from .. import k8s
from ..k8s import V1Container, V1ResourceRequirements, V1VolumeMount
from . import _pipeline_param
from ._metadata import ComponentMeta
from ._pipeline_volume import PipelineVolume


def as_string_list(list_or_str) -> list | None:
    if list_or_str is None:
        return None
    if isinstance(list_or_str, (list, tuple)):
        return [str(x) for x in list_or_str]
    return [str(list_or_str)]


def create_and_append(current_list, item):
    current_list = current_list or []
    current_list.append(item)
    return current_list


class Container(V1Container):
    """`io.argoproj.workflow.v1alpha1.Template.container` with fluent resource/env/volume helpers."""

    swagger_types = {k: v for k, v in V1Container.swagger_types.items() if k != "name"}
    attribute_map = {k: v for k, v in V1Container.attribute_map.items() if k != "name"}

    def __init__(self, image: str, command, args, **kwargs):
        name = kwargs.pop("name", "") or ""
        super().__init__(image=image, command=command, args=args, **kwargs)
        self.name = name

    # ---- validators --------------------------------------------------------------------------
    @staticmethod
    def _validate_memory_string(memory_string):
        if re.match(r"^[0-9]+(E|Ei|P|Pi|T|Ti|G|Gi|M|Mi|K|Ki){0,1}$", memory_string) is None:
            raise ValueError('Invalid memory string. Should be an integer, or integer followed by one of '
                             '"E|Ei|P|Pi|T|Ti|G|Gi|M|Mi|K|Ki"')

    @staticmethod
    def _validate_cpu_string(cpu_string):
        if re.match(r"^[0-9]+m$", cpu_string) is not None:
            return
        try:
            float(cpu_string)
        except ValueError as e:
            raise ValueError('Invalid cpu string. Should be float or integer, or integer followed by "m".') from e

    @staticmethod
    def _validate_positive_number(str_value, param_name):
        try:
            v = int(str_value)
        except ValueError as e:
            raise ValueError(f"Invalid {param_name}. Should be integer.") from e
        if v <= 0:
            raise ValueError(f"{param_name} must be positive integer.")

    # ---- resources ---------------------------------------------------------------------------
    def add_resource_limit(self, resource_name, value):
        self.resources = self.resources or V1ResourceRequirements()
        self.resources.limits = self.resources.limits or {}
        self.resources.limits.update({resource_name: value})
        return self

    def add_resource_request(self, resource_name, value):
        self.resources = self.resources or V1ResourceRequirements()
        self.resources.requests = self.resources.requests or {}
        self.resources.requests.update({resource_name: value})
        return self

    def set_memory_request(self, memory):
        self._validate_memory_string(memory)
        return self.add_resource_request("memory", memory)

    def set_memory_limit(self, memory):
        self._validate_memory_string(memory)
        return self.add_resource_limit("memory", memory)

    def set_cpu_request(self, cpu):
        self._validate_cpu_string(cpu)
        return self.add_resource_request("cpu", cpu)

    def set_cpu_limit(self, cpu):
        self._validate_cpu_string(cpu)
        return self.add_resource_limit("cpu", cpu)

    def set_gpu_limit(self, gpu, vendor: str = "nvidia"):
        self._validate_positive_number(gpu, "gpu")
        if vendor not in ("nvidia", "amd"):
            raise ValueError("vendor can only be nvidia or amd.")
        return self.add_resource_limit(f"{vendor}.com/gpu", gpu)

    # ---- misc container fields ---------------------------------------------------------------
    def add_volume_mount(self, volume_mount):
        if not isinstance(volume_mount, V1VolumeMount):
            raise ValueError("invalid argument. Must be of instance `V1VolumeMount`.")
        self.volume_mounts = create_and_append(self.volume_mounts, volume_mount)
        return self

    def add_volume_devices(self, volume_device):
        self.volume_devices = create_and_append(self.volume_devices, volume_device)
        return self

    def add_env_variable(self, env_variable):
        if not isinstance(env_variable, k8s.V1EnvVar):
            raise ValueError("invalid argument. Must be of instance `V1EnvVar`.")
        self.env = create_and_append(self.env, env_variable)
        return self

    def add_env_from(self, env_from):
        self.env_from = create_and_append(self.env_from, env_from)
        return self

    def set_image_pull_policy(self, image_pull_policy):
        if image_pull_policy not in ("Always", "Never", "IfNotPresent"):
            raise ValueError("Invalid imagePullPolicy. Must be one of `Always`, `Never`, `IfNotPresent`.")
        self.image_pull_policy = image_pull_policy
        return self

    def add_port(self, container_port):
        self.ports = create_and_append(self.ports, container_port)
        return self

    def set_security_context(self, security_context):
        self.security_context = security_context
        return self

    def set_stdin(self, stdin=True):
        self.stdin = stdin
        return self

    def set_stdin_once(self, stdin_once=True):
        self.stdin_once = stdin_once
        return self

    def set_termination_message_path(self, termination_message_path):
        self.termination_message_path = termination_message_path
        return self

    def set_termination_message_policy(self, termination_message_policy):
        if termination_message_policy not in ("File", "FallbackToLogsOnError"):
            raise ValueError("terminationMessagePolicy must be `File` or `FallbackToLogsOnError`")
        self.termination_message_policy = termination_message_policy
        return self

    def set_tty(self, tty=True):
        self.tty = tty
        return self

    def set_readiness_probe(self, readiness_probe):
        self.readiness_probe = readiness_probe
        return self

    def set_liveness_probe(self, liveness_probe):
        self.liveness_probe = liveness_probe
        return self

    def set_lifecycle(self, lifecycle):
        self.lifecycle = lifecycle
        return self


class Sidecar(Container):
    swagger_types = dict(V1Container.swagger_types, mirror_volume_mounts="bool")
    attribute_map = dict(V1Container.attribute_map, mirror_volume_mounts="mirrorVolumeMounts")

    def __init__(self, name: str, image: str, command=None, args=None, mirror_volume_mounts: bool | None = None,
                 **kwargs):
        super().__init__(image=image, command=as_string_list(command), args=as_string_list(args), name=name,
                         **kwargs)
        self.mirror_volume_mounts = mirror_volume_mounts

    def set_mirror_volume_mounts(self, mirror_volume_mounts=True):
        self.mirror_volume_mounts = mirror_volume_mounts
        return self

    @property
    def inputs(self):
        return _pipeline_param.extract_pipelineparams_from_any(self)


def _make_hash_based_id_for_op(op) -> str:
    return op.human_name + " " + hex(2 ** 63 + hash(op))[2:]


# replaced by the active Pipeline context to register ops and make names unique
_register_op_handler: Callable = _make_hash_based_id_for_op


class BaseOp:
    attrs_with_pipelineparams = ["node_selector", "volumes", "pod_annotations", "pod_labels", "num_retries",
                                 "sidecars", "tolerations"]

    def __init__(self, name: str, sidecars=None, is_exit_handler: bool = False):
        if not re.match(r"^[A-Za-z][A-Za-z0-9\s_-]*$", name):
            raise ValueError('Only letters, numbers, spaces, "_", and "-"  are allowed in name. Must begin with '
                             f"letter: {name}")
        self.is_exit_handler = is_exit_handler
        self.human_name = name
        self.display_name = None
        from . import _container_op as me  # late lookup: the Pipeline context swaps the handler

        self.name = me._register_op_handler(self)
        self.node_selector = {}
        self.volumes = []
        self.tolerations = []
        self.pod_annotations = {}
        self.pod_labels = {}
        self.num_retries = 0
        self.timeout = 0
        self.sidecars = sidecars or []
        self._inputs = []
        self.dependent_names = []

    @property
    def inputs(self):
        if not self._inputs:
            found = []
            for key in self.attrs_with_pipelineparams:
                found += _pipeline_param.extract_pipelineparams_from_any(getattr(self, key))
            self._inputs = list(dict.fromkeys(found))
        return self._inputs

    @inputs.setter
    def inputs(self, value):
        self._inputs = value

    def apply(self, mod_func):
        return mod_func(self) or self

    def after(self, *ops):
        for op in ops:
            self.dependent_names.append(op.name)
        return self

    def add_volume(self, volume):
        self.volumes.append(volume)
        return self

    def add_toleration(self, tolerations):
        self.tolerations.append(tolerations)
        return self

    def add_node_selector_constraint(self, label_name, value):
        self.node_selector[label_name] = value
        return self

    def add_pod_annotation(self, name: str, value: str):
        self.pod_annotations[name] = value
        return self

    def add_pod_label(self, name: str, value: str):
        self.pod_labels[name] = value
        return self

    def set_retry(self, num_retries: int):
        self.num_retries = num_retries
        return self

    def set_timeout(self, seconds: int):
        self.timeout = seconds
        return self

    def add_sidecar(self, sidecar):
        self.sidecars.append(sidecar)
        return self

    def set_display_name(self, name: str):
        self.display_name = name
        return self

    def __repr__(self):
        return str({type(self).__name__: self.__dict__})


class ContainerOp(BaseOp):
    """A step running a container image with arguments, file outputs and volumes."""

    _NO_PROXY = frozenset(["to_dict", "to_str"])

    def __init__(self, name: str, image: str, command=None, arguments=None, sidecars=None,
                 container_kwargs: dict | None = None, file_outputs: dict | None = None,
                 output_artifact_paths: dict | None = None, artifact_location=None, is_exit_handler: bool = False,
                 pvolumes: dict | None = None):
        super().__init__(name=name, sidecars=sidecars, is_exit_handler=is_exit_handler)
        self.attrs_with_pipelineparams = BaseOp.attrs_with_pipelineparams + ["_container", "artifact_location"]
        self._container = Container(image=image, args=as_string_list(arguments), command=as_string_list(command),
                                    **(container_kwargs or {}))
        self.file_outputs = file_outputs
        self.output_artifact_paths = output_artifact_paths or {}
        self.artifact_location = artifact_location
        self._metadata = None
        self.outputs = {}
        if file_outputs:
            self.outputs = {n: _pipeline_param.PipelineParam(n, op_name=self.name) for n in file_outputs}
        self.output = list(self.outputs.values())[0] if len(self.outputs) == 1 else None
        self.pvolumes = {}
        self.add_pvolumes(pvolumes)

    def __getattr__(self, item):
        # proxy Container helper methods (deprecated in the reference but still supported there)
        if item.startswith("_") or item in self._NO_PROXY:
            raise AttributeError(item)
        cont = self.__dict__.get("_container")
        attr = getattr(cont, item, None) if cont is not None else None
        if callable(attr):
            def _proxy(*args, **kwargs):
                warnings.warn(f"ContainerOp.{item} is deprecated, use ContainerOp.container.{item}",
                              PendingDeprecationWarning, stacklevel=2)
                ret = attr(*args, **kwargs)
                return self if ret is cont else ret

            return _proxy
        raise AttributeError(item)

    @property
    def command(self):
        return self._container.command

    @command.setter
    def command(self, value):
        self._container.command = as_string_list(value)

    @property
    def arguments(self):
        return self._container.args

    @arguments.setter
    def arguments(self, value):
        self._container.args = as_string_list(value)

    @property
    def container(self) -> Container:
        return self._container

    # deprecated property proxies onto the container (reference `_container_op.py:51-83`: image, env_variables)
    def _deprecated(self, prop: str, target: str):
        warnings.warn(f"`dsl.ContainerOp.{prop}` will be removed in future releases. "
                      f"Use `dsl.ContainerOp.container.{target}` instead.", PendingDeprecationWarning, stacklevel=3)

    @property
    def image(self):
        self._deprecated("image", "image")
        return self._container.image

    @image.setter
    def image(self, value):
        self._deprecated("image", "image")
        self._container.image = value

    @property
    def env_variables(self):
        self._deprecated("env_variables", "env")
        return self._container.env

    @env_variables.setter
    def env_variables(self, value):
        self._deprecated("env_variables", "env")
        self._container.env = value

    def _set_metadata(self, metadata: ComponentMeta):
        if not isinstance(metadata, ComponentMeta):
            raise ValueError("_set_metadata is expecting ComponentMeta.")
        self._metadata = metadata
        if self.file_outputs:
            for out in self.file_outputs:
                t = self.outputs[out].param_type
                for om in metadata.outputs:
                    if om.name == out:
                        t = om.param_type
                self.outputs[out].param_type = t
            self.output = list(self.outputs.values())[0] if len(self.outputs) == 1 else None

    def add_pvolumes(self, pvolumes: dict | None = None):
        if pvolumes:
            for mount_path, pvolume in pvolumes.items():
                if hasattr(pvolume, "dependent_names"):
                    self.dependent_names.extend(pvolume.dependent_names)
                else:
                    pvolume = PipelineVolume(volume=pvolume)
                self.pvolumes[mount_path] = pvolume.after(self)
                self.add_volume(pvolume)
                self._container.add_volume_mount(V1VolumeMount(name=pvolume.name, mount_path=mount_path))
        self.pvolume = list(self.pvolumes.values())[0] if len(self.pvolumes) == 1 else None
        return self
