"""component.yaml schema: ComponentSpec, ContainerSpec, placeholders, graph components.

Reference: `sdk/python/kfp/components/_structures.py:68-554` — inputs/outputs, container
implementation with command/args placeholders (`inputValue`, `inputPath`, `outputPath`, `concat`,
`if`/`isPresent`), `fileOutputs`, graph implementation (tasks with componentRef/arguments/
isEnabled predicates, outputValues) with topological-sort cycle detection, and validation that
every placeholder references a declared input/output."""
from __future__ import annotations

from collections import OrderedDict
from typing import Any, Dict, List, Mapping, Optional, Union

from .modelbase import ModelBase
from .structures.kubernetes import v1 as k8s_v1

PrimitiveTypes = Union[str, int, float, bool]
PrimitiveTypesIncludingNone = Optional[PrimitiveTypes]
TypeType = Union[str, Dict, List]


class InputSpec(ModelBase):
    def __init__(self, name: str, type: Optional[TypeType] = None, description: Optional[str] = None,  # noqa: A002
                 default: Optional[PrimitiveTypes] = None, optional: Optional[bool] = False):
        self.name = name
        self.type = type
        self.description = description
        self.default = default
        self.optional = optional

    def to_dict(self):
        d = super().to_dict()
        if d.get("optional") is False:
            d.pop("optional")
        return d


class OutputSpec(ModelBase):
    def __init__(self, name: str, type: Optional[TypeType] = None, description: Optional[str] = None):  # noqa: A002
        self.name = name
        self.type = type
        self.description = description


class InputValuePlaceholder(ModelBase):
    _serialized_names = {"input_name": "inputValue"}

    def __init__(self, input_name: str):
        self.input_name = input_name


class InputPathPlaceholder(ModelBase):
    _serialized_names = {"input_name": "inputPath"}

    def __init__(self, input_name: str):
        self.input_name = input_name


class OutputPathPlaceholder(ModelBase):
    _serialized_names = {"output_name": "outputPath"}

    def __init__(self, output_name: str):
        self.output_name = output_name


CommandlineArgumentType = Union[str, InputValuePlaceholder, InputPathPlaceholder, OutputPathPlaceholder,
                                "ConcatPlaceholder", "IfPlaceholder"]


class ConcatPlaceholder(ModelBase):
    _serialized_names = {"items": "concat"}

    def __init__(self, items: List[CommandlineArgumentType]):
        self.items = items


class IsPresentPlaceholder(ModelBase):
    _serialized_names = {"input_name": "isPresent"}

    def __init__(self, input_name: str):
        self.input_name = input_name


IfConditionArgumentType = Union[bool, str, IsPresentPlaceholder, InputValuePlaceholder]


class IfPlaceholderStructure(ModelBase):
    _serialized_names = {"condition": "cond", "then_value": "then", "else_value": "else"}

    def __init__(self, condition: IfConditionArgumentType,
                 then_value: Union[CommandlineArgumentType, List[CommandlineArgumentType]],
                 else_value: Optional[Union[CommandlineArgumentType, List[CommandlineArgumentType]]] = None):
        self.condition = condition
        self.then_value = then_value
        self.else_value = else_value


class IfPlaceholder(ModelBase):
    _serialized_names = {"if_structure": "if"}

    def __init__(self, if_structure: IfPlaceholderStructure):
        self.if_structure = if_structure


class ContainerSpec(ModelBase):
    _serialized_names = {"file_outputs": "fileOutputs"}

    def __init__(self, image: str, command: Optional[List[CommandlineArgumentType]] = None,
                 args: Optional[List[CommandlineArgumentType]] = None, env: Optional[Mapping[str, str]] = None,
                 file_outputs: Optional[Mapping[str, str]] = None):
        self.image = image
        self.command = command
        self.args = args
        self.env = env
        self.file_outputs = file_outputs


class ContainerImplementation(ModelBase):
    def __init__(self, container: ContainerSpec):
        self.container = container


class MetadataSpec(ModelBase):
    def __init__(self, annotations: Optional[Dict[str, str]] = None, labels: Optional[Dict[str, str]] = None):
        self.annotations = annotations
        self.labels = labels


# ----------------------------------------------------------------------------- graph
class GraphInputArgument(ModelBase):
    _serialized_names = {"input_name": "graphInput"}

    def __init__(self, input_name: str):
        self.input_name = input_name


class TaskOutputReference(ModelBase):
    _serialized_names = {"task_id": "taskId", "output_name": "outputName"}

    def __init__(self, output_name: str, task_id: Optional[str] = None, task: Optional["TaskSpec"] = None):
        self.output_name = output_name
        self.task_id = task_id
        self.task = task

    def to_dict(self):
        d = {"outputName": self.output_name}
        if self.task_id is not None:
            d["taskId"] = self.task_id
        return d


class TaskOutputArgument(ModelBase):
    _serialized_names = {"task_output": "taskOutput"}

    def __init__(self, task_output: TaskOutputReference):
        self.task_output = task_output

    @staticmethod
    def construct(task_id: str, output_name: str) -> "TaskOutputArgument":
        return TaskOutputArgument(TaskOutputReference(task_id=task_id, output_name=output_name))


ArgumentType = Union[PrimitiveTypes, GraphInputArgument, TaskOutputArgument]


class TwoOperands(ModelBase):
    def __init__(self, op1: ArgumentType, op2: ArgumentType):
        self.op1 = op1
        self.op2 = op2


class BinaryPredicate(ModelBase):
    def __init__(self, operands: TwoOperands):
        self.operands = operands


class EqualsPredicate(BinaryPredicate):
    _serialized_names = {"operands": "=="}


class NotEqualsPredicate(BinaryPredicate):
    _serialized_names = {"operands": "!="}


class GreaterThanPredicate(BinaryPredicate):
    _serialized_names = {"operands": ">"}


class GreaterThanOrEqualPredicate(BinaryPredicate):
    _serialized_names = {"operands": ">="}


class LessThenPredicate(BinaryPredicate):
    _serialized_names = {"operands": "<"}


class LessThenOrEqualPredicate(BinaryPredicate):
    _serialized_names = {"operands": "<="}


class TwoBooleanOperands(ModelBase):
    def __init__(self, op1: "PredicateType", op2: "PredicateType"):
        self.op1 = op1
        self.op2 = op2


class NotPredicate(ModelBase):
    _serialized_names = {"operand": "not"}

    def __init__(self, operand: "PredicateType"):
        self.operand = operand


class AndPredicate(ModelBase):
    _serialized_names = {"operands": "and"}

    def __init__(self, operands: TwoBooleanOperands):
        self.operands = operands


class OrPredicate(ModelBase):
    _serialized_names = {"operands": "or"}

    def __init__(self, operands: TwoBooleanOperands):
        self.operands = operands


PredicateType = Union[ArgumentType, EqualsPredicate, NotEqualsPredicate, GreaterThanPredicate,
                      GreaterThanOrEqualPredicate, LessThenOrEqualPredicate, LessThenPredicate, NotPredicate,
                      AndPredicate, OrPredicate]


class ExecutionOptionsSpec(ModelBase):
    _serialized_names = {"retry_strategy": "retryStrategy", "active_deadline_seconds": "activeDeadlineSeconds"}

    def __init__(self, retry_strategy: Optional[Dict[str, Any]] = None, active_deadline_seconds: Optional[int] = None):
        self.retry_strategy = retry_strategy
        self.active_deadline_seconds = active_deadline_seconds


class ComponentReference(ModelBase):
    def __init__(self, name: Optional[str] = None, digest: Optional[str] = None, tag: Optional[str] = None,
                 url: Optional[str] = None, spec: Optional["ComponentSpec"] = None):
        self.name = name
        self.digest = digest
        self.tag = tag
        self.url = url
        self.spec = spec
        if not any((name, digest, tag, url, spec)):
            raise TypeError("Need at least one argument.")


class TaskSpec(ModelBase):
    _serialized_names = {"component_ref": "componentRef", "is_enabled": "isEnabled",
                         "execution_options": "executionOptions", "k8s_container_options": "k8sContainerOptions",
                         "k8s_pod_options": "k8sPodOptions"}

    def __init__(self, component_ref: ComponentReference, arguments: Optional[Mapping[str, ArgumentType]] = None,
                 is_enabled: Optional[PredicateType] = None, execution_options: Optional[ExecutionOptionsSpec] = None,
                 k8s_container_options: Optional[k8s_v1.Container] = None,
                 k8s_pod_options: Optional[k8s_v1.PodArgoSubset] = None):
        self.component_ref = component_ref
        self.arguments = arguments
        self.is_enabled = is_enabled
        self.execution_options = execution_options
        self.k8s_container_options = k8s_container_options
        self.k8s_pod_options = k8s_pod_options


class GraphSpec(ModelBase):
    _serialized_names = {"output_values": "outputValues"}

    def __init__(self, tasks: Mapping[str, TaskSpec], output_values: Optional[Mapping[str, ArgumentType]] = None):
        self.tasks = tasks
        self.output_values = output_values
        self._toposorted_tasks = self._toposort()

    def _toposort(self) -> "OrderedDict[str, TaskSpec]":
        """Depth-first topological order of tasks; raises on dependency cycles."""
        deps = {}
        for tid, task in self.tasks.items():
            d = set()
            for arg in (task.arguments or {}).values():
                if isinstance(arg, TaskOutputArgument):
                    ref = arg.task_output.task_id
                    if ref not in self.tasks:
                        raise TypeError(f"Argument of task {tid} references non-existing task {ref}.")
                    d.add(ref)
            deps[tid] = d
        order, state = OrderedDict(), {}

        def visit(t):
            s = state.get(t)
            if s == 1:
                raise ValueError(f"Task {t} has a dependency cycle.")
            if s == 2:
                return
            state[t] = 1
            for u in sorted(deps[t]):
                visit(u)
            state[t] = 2
            order[t] = self.tasks[t]

        for t in self.tasks:
            visit(t)
        return order


class GraphImplementation(ModelBase):
    def __init__(self, graph: GraphSpec):
        self.graph = graph


ImplementationType = Union[ContainerImplementation, GraphImplementation]


class ComponentSpec(ModelBase):
    def __init__(self, name: Optional[str] = None, description: Optional[str] = None,
                 metadata: Optional[MetadataSpec] = None, inputs: Optional[List[InputSpec]] = None,
                 outputs: Optional[List[OutputSpec]] = None, implementation: Optional[ImplementationType] = None,
                 version: Optional[str] = "google.com/cloud/pipelines/component/v1"):
        self.name = name
        self.description = description
        self.metadata = metadata
        self.inputs = inputs
        self.outputs = outputs
        self.implementation = implementation
        self.version = version
        self._validate()

    def _validate(self):
        ins = {i.name for i in self.inputs or []}
        outs = {o.name for o in self.outputs or []}
        if len(ins) != len(self.inputs or []):
            raise ValueError("Non-unique input names.")
        if len(outs) != len(self.outputs or []):
            raise ValueError("Non-unique output names.")
        impl = self.implementation
        if isinstance(impl, ContainerImplementation):
            c = impl.container
            if c.file_outputs:
                for name in c.file_outputs:
                    if name not in outs:
                        raise TypeError(f'Unconfigurable output entry "{name}" references non-existing output.')

            def check(arg):
                if arg is None or isinstance(arg, (str, int, float, bool)):
                    return
                if isinstance(arg, list):
                    for a in arg:
                        check(a)
                elif isinstance(arg, (InputValuePlaceholder, InputPathPlaceholder, IsPresentPlaceholder)):
                    if arg.input_name not in ins:
                        raise TypeError(f'Argument "{arg}" references non-existing input.')
                elif isinstance(arg, OutputPathPlaceholder):
                    if arg.output_name not in outs:
                        raise TypeError(f'Argument "{arg}" references non-existing output.')
                elif isinstance(arg, ConcatPlaceholder):
                    for a in arg.items:
                        check(a)
                elif isinstance(arg, IfPlaceholder):
                    s = arg.if_structure
                    check(s.condition)
                    check(s.then_value)
                    check(s.else_value)
                else:
                    raise TypeError(f"Unexpected argument {arg!r}")

            for a in (c.command or []) + (c.args or []):
                check(a)
        elif isinstance(impl, GraphImplementation):
            g = impl.graph
            for tid, task in g.tasks.items():
                for arg in (task.arguments or {}).values():
                    if isinstance(arg, GraphInputArgument) and arg.input_name not in ins:
                        raise TypeError(f'Argument "{arg}" references non-existing input.')
            for name in (g.output_values or {}):
                if name not in outs:
                    raise TypeError(f'Output value "{name}" references non-existing output.')


class PipelineRunSpec(ModelBase):
    _serialized_names = {"pipeline_spec": "pipelineSpec"}

    def __init__(self, pipeline_spec: ComponentSpec, arguments: Optional[Mapping[str, ArgumentType]] = None):
        self.pipeline_spec = pipeline_spec
        self.arguments = arguments
