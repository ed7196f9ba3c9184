"""component.yaml loading, task-factory signatures, placeholder expansion, type compatibility,
graph components and the typed ModelBase.

Mirrors the reference strategy of `sdk/python/tests/components/{test_components,test_graph_components,
test_structure_model_base}.py`: each case is a small component.yaml text loaded through the
public loaders; the produced ContainerOp's command/arguments/env/metadata are the observable result.
"""
import inspect
import zipfile
from typing import Dict, List, Optional, Union

import pytest

import mifx.kfp as kfp
from mifx.kfp import components as comp
from mifx.kfp.components._structures import (ComponentReference, ComponentSpec, GraphImplementation,
                                             GraphInputArgument, GraphSpec, InputSpec, OutputSpec,
                                             TaskOutputArgument, TaskSpec)
from mifx.kfp.components._yaml_utils import load_yaml
from mifx.kfp.components.modelbase import ModelBase
from mifx.kfp.dsl import Pipeline
from mifx.kfp.dsl.types import InconsistentTypeException

BUSYBOX = "implementation:\n  container:\n    image: busybox\n"


def _load(text):
    return comp.load_component_from_text(text)


@pytest.fixture(autouse=True)
def _type_check_on():
    prev = kfp.TYPE_CHECK
    kfp.TYPE_CHECK = True
    yield
    kfp.TYPE_CHECK = prev


# ---------------------------------------------------------------- loaders (_components.py:35-127)

def test_minimal_component_and_file_zip_loaders(tmp_path):
    f = tmp_path / "component.yaml"
    f.write_text("name: Tiny\n" + BUSYBOX)
    z = tmp_path / "component.zip"
    with zipfile.ZipFile(z, "w") as zf:
        zf.writestr("component.yaml", f.read_text())
    for factory in (comp.load_component(text=BUSYBOX), comp.load_component_from_file(str(f)),
                    comp.load_component_from_file(str(z)), comp.load_component(filename=str(f))):
        assert factory().container.image == "busybox"


@pytest.mark.parametrize("call", [
    lambda: comp.load_component(),
    lambda: comp.load_component(filename="", text=""),
    lambda: comp.load_component(filename=None, url=None, text=None),
    lambda: comp.load_component_from_file(None),
    lambda: comp.load_component_from_url(None),
    lambda: comp.load_component_from_text(None),
])
def test_loader_argument_errors(call):
    with pytest.raises((ValueError, TypeError)):
        call()


@pytest.mark.parametrize("text", [
    "inputs:\n- {name: Data1}\n- {name: Data1}\n" + BUSYBOX,
    "outputs:\n- {name: Data1}\n- {name: Data1}\n" + BUSYBOX,
    "inputs:\n- {name: Data}\n" + BUSYBOX + "    args:\n      - {inputValue: Wrong}\n",
    "outputs:\n- {name: Data}\n" + BUSYBOX + "    fileOutputs:\n      Wrong: /outputs/output.txt\n",
])
def test_invalid_specs_are_rejected(text):
    with pytest.raises(Exception):
        _load(text)


@pytest.mark.parametrize("text", [
    "inputs:\n- {name: Data}\n- {name: _Data}\n" + BUSYBOX,
    "outputs:\n- {name: Data}\n- {name: _Data}\n" + BUSYBOX,
    "inputs:\n- {name: Training data}\n" + BUSYBOX,
    "outputs:\n- {name: Training data}\n" + BUSYBOX,
    "outputs:\n- {name: Output data}\n" + BUSYBOX + "    fileOutputs:\n      Output data: /outputs/output-data\n",
    "inputs:\n- {name: Input 1}\n- {name: Input_1}\n- {name: Input-1}\n" + BUSYBOX,
    "inputs:\n- {name: Data}\noutputs:\n- {name: Data}\n" + BUSYBOX,
])
def test_awkward_but_valid_names_load_and_instantiate(text):
    factory = _load(text)
    params = list(inspect.signature(factory).parameters)
    assert len(params) == len(set(params))  # pythonic names are made unique
    task = factory(*["v"] * sum(1 for p in inspect.signature(factory).parameters.values()
                                if p.default is inspect.Parameter.empty))
    assert task.container.image == "busybox"


# ---------------------------------------------------------------- task factory signature (_components.py:197-256)

@pytest.mark.parametrize("inputs,order", [
    ("- {name: in1}\n- {name: in2, optional: true}\n- {name: in3}\n", ["in1", "in3", "in2"]),
    ("- {name: in1}\n- {name: in2, default: val}\n- {name: in3}\n", ["in1", "in3", "in2"]),
    ("- {name: a1}\n- {name: b1, default: val}\n- {name: a2}\n- {name: b2, optional: True}\n- {name: a3}\n"
     "- {name: b3, default: val}\n- {name: a4}\n- {name: b4, optional: True}\n",
     ["a1", "a2", "a3", "a4", "b1", "b2", "b3", "b4"]),
])
def test_required_inputs_come_first_and_order_is_stable(inputs, order):
    assert list(inspect.signature(_load("inputs:\n" + inputs + BUSYBOX)).parameters) == order


def test_default_values_in_task_factory():
    f = _load("inputs:\n- {name: Data, default: '123'}\n" + BUSYBOX + "    args:\n      - {inputValue: Data}\n")
    assert f().arguments == ["123"]
    assert f("456").arguments == ["456"]


# ---------------------------------------------------------------- placeholders (_dsl_bridge.py:37-118)

def test_input_value_and_output_path_resolution():
    f = _load("inputs:\n- {name: Data}\noutputs:\n- {name: Out}\n" + BUSYBOX +
              "    args:\n      - --data\n      - inputValue: Data\n      - --out\n      - {outputPath: Out}\n")
    task = f("some-data")
    assert task.arguments[:3] == ["--data", "some-data", "--out"]
    assert task.arguments[3].startswith("/")
    assert task.file_outputs == {"out": task.arguments[3]}  # output names are k8s-sanitised


@pytest.mark.parametrize("placeholder", ["inputValue", "inputPath"])
def test_missing_optional_input_resolves_to_nothing(placeholder):
    f = _load("inputs:\n- {name: input 1, optional: true}\n" + BUSYBOX +
              f"    command:\n      - a\n      - {{{placeholder}: input 1}}\n      - z\n")
    assert f().command == ["a", "z"]


def test_concat_placeholder():
    f = _load("inputs:\n- {name: In1}\n- {name: In2}\n" + BUSYBOX +
              "    args:\n      - concat: [{inputValue: In1}, '-', {inputValue: In2}]\n")
    assert f("some", "data").arguments == ["some-data"]


@pytest.mark.parametrize("cond,want", [("true", "--true-arg"), ("false", "--false-arg"),
                                       ("'true'", "--true-arg"), ("'false'", "--false-arg")])
def test_if_placeholder_with_constant_condition(cond, want):
    f = _load(BUSYBOX + f"    args:\n      - if:\n          cond: {cond}\n          then: --true-arg\n"
                        f"          else: --false-arg\n")
    assert f().arguments == [want]


@pytest.mark.parametrize("with_else", [False, True])
def test_if_is_present_placeholder(with_else):
    text = ("inputs:\n- {name: In, optional: true}\n" + BUSYBOX +
            "    args:\n      - if:\n          cond: {isPresent: In}\n          then: [--in, {inputValue: In}]\n")
    if with_else:
        text += "          else: --no-in\n"
    f = _load(text)
    assert f("data").arguments == ["--in", "data"]
    assert f().arguments == (["--no-in"] if with_else else [])


def test_if_on_boolean_input_value():
    f = _load("inputs:\n- {name: Do test, type: boolean, optional: true}\n- {name: Test data, optional: true}\n"
              "- {name: Test parameter 1, optional: true}\n" + BUSYBOX +
              "    args:\n      - if:\n          cond: {inputValue: Do test}\n"
              "          then: [--test-data, {inputValue: Test data}, --test-param1, {inputValue: Test parameter 1}]\n")
    assert f(True, "test_data.txt", 42).arguments == ["--test-data", "test_data.txt", "--test-param1", "42"]
    assert f().arguments == []


def test_env_and_metadata_reach_the_container_op():
    f = _load("metadata:\n  annotations:\n    a1: v1\n  labels:\n    l1: v2\n" + BUSYBOX +
              "    env:\n      key1: value 1\n      key2: value 2\n")
    task = f()
    assert {e.name: e.value for e in task.container.env} == {"key1": "value 1", "key2": "value 2"}
    assert task.pod_annotations["a1"] == "v1" and task.pod_labels["l1"] == "v2"


# ---------------------------------------------------------------- type compatibility (_components.py:188-256)

_PRODUCER = ("outputs:\n  - {{name: out1{t}}}\n" + BUSYBOX +
             "    command: [sh, -c, 'date > \"$0\"', {{outputPath: out1}}]\n")
_CONSUMER = "inputs:\n  - {{name: in1{t}}}\n" + BUSYBOX + "    command: [echo, {{inputValue: in1}}]\n"
_GCS = "{GCSPath: {openapi_schema_validator: {type: string, pattern: %s}}}"


@pytest.mark.parametrize("out_t,in_t,ok", [
    ("custom_type", "custom_type", True),
    ("{parametrized_type: {property_a: value_a, property_b: value_b}}",
     "{parametrized_type: {property_a: value_a, property_b: value_b}}", True),
    ("custom_type", None, True),            # input type missing: anything goes
    (None, "custom_type", True),            # argument type missing: anything goes
    ("type_A", "type_Z", False),
    ("{parametrized_type_A: {property_a: value_a}}", "{parametrized_type_Z: {property_a: value_a}}", False),
    ("{parametrized_type: {property_a: value_a}}", "{parametrized_type: {property_a: DIFFERENT}}", False),
    (_GCS % '"^gs://.*$"', _GCS % '"^gs://.*$"', True),
    (_GCS % "AAA", _GCS % "ZZZ", False),
])
@pytest.mark.parametrize("positional", [False, True])
def test_type_compatibility(out_t, in_t, ok, positional):
    a = _load(_PRODUCER.format(t="" if out_t is None else f", type: {out_t}"))
    b = _load(_CONSUMER.format(t="" if in_t is None else f", type: {in_t}"))
    with Pipeline("types"):
        out = a().outputs["out1"]

        def wire(arg):
            return b(arg) if positional else b(in1=arg)

        if ok:
            wire(out)
        else:
            with pytest.raises(InconsistentTypeException):
                wire(out)
            wire(out.ignore_type())  # explicit opt-out
            kfp.TYPE_CHECK = False   # global opt-out
            wire(out)


# ---------------------------------------------------------------- graph components (_structures.py:466-533)

def test_construct_graph_component_in_code():
    t1 = TaskSpec(component_ref=ComponentReference(name="comp 1"), arguments={"in1 1": 11})
    t2 = TaskSpec(component_ref=ComponentReference(name="comp 2"), arguments={
        "in2 1": 21, "in2 2": TaskOutputArgument.construct(task_id="task 1", output_name="out1 1")})
    t3 = TaskSpec(component_ref=ComponentReference(name="comp 3"), arguments={
        "in3 1": TaskOutputArgument.construct(task_id="task 2", output_name="out2 1"),
        "in3 2": GraphInputArgument(input_name="graph in 1")})
    spec = ComponentSpec(
        inputs=[InputSpec(name="graph in 1"), InputSpec(name="graph in 2")],
        outputs=[OutputSpec(name="graph out 1"), OutputSpec(name="graph out 2")],
        implementation=GraphImplementation(graph=GraphSpec(
            tasks={"task 1": t1, "task 2": t2, "task 3": t3},
            output_values={"graph out 1": TaskOutputArgument.construct(task_id="task 3", output_name="out3 1"),
                           "graph out 2": TaskOutputArgument.construct(task_id="task 1", output_name="out1 2")})))
    again = ComponentSpec.from_dict(spec.to_dict())
    assert list(again.implementation.graph.tasks) == ["task 1", "task 2", "task 3"]


_GRAPH = """\
inputs:
- {name: graph in 1}
outputs:
- {name: graph out 1}
implementation:
  graph:
    tasks:
      task 1:
        componentRef: {name: Comp 1}
        arguments:
            in1 1: 11
      task 2:
        componentRef: {name: Comp 2}
        arguments:
            in2 1: {taskOutput: {taskId: task 1, outputName: out1 1}}
            in2 2: {graphInput: graph in 1}
        isEnabled:
            not:
                and:
                    op1: {'>': {op1: {taskOutput: {taskId: task 1, outputName: out1 1}}, op2: 0}}
                    op2: {'==': {op1: {taskOutput: {taskId: task 1, outputName: out1 2}}, op2: head}}
        k8sContainerOptions:
          resources:
            requests: {memory: 1024Mi, cpu: 200m}
          volumeMounts:
          - {name: workdir, mountPath: /mnt/vol}
        k8sPodOptions:
          spec:
            volumes:
            - {name: workdir, emptyDir: {}}
    outputValues:
      graph out 1: {taskOutput: {taskId: task 2, outputName: out2 1}}
"""


def test_parse_graph_component_with_predicates_and_k8s_options():
    spec = ComponentSpec.from_dict(load_yaml(_GRAPH))
    t2 = spec.implementation.graph.tasks["task 2"]
    assert t2.k8s_container_options.resources.requests["memory"] == "1024Mi"
    assert t2.k8s_pod_options.spec.volumes[0].name == "workdir"
    assert t2.k8s_pod_options.spec.volumes[0].empty_dir is not None
    assert t2.is_enabled is not None


def test_cyclic_task_references_are_rejected():
    text = """\
implementation:
  graph:
    tasks:
      task 1:
        componentRef: {name: Comp 1}
        arguments:
            in1 1: {taskOutput: {taskId: task 2, outputName: out2 1}}
      task 2:
        componentRef: {name: Comp 2}
        arguments:
            in2 1: {taskOutput: {taskId: task 1, outputName: out1 1}}
"""
    with pytest.raises(Exception):
        ComponentSpec.from_dict(load_yaml(text))


# ---------------------------------------------------------------- ModelBase (modelbase.py:95-287)

class _Model(ModelBase):
    _serialized_names = {"prop_1": "prop1", "prop_2": "prop 2", "prop_3": "@@"}

    def __init__(self, prop_0: str, prop_1: Optional[str] = None, prop_2: Union[int, str, bool] = "",
                 prop_3: "_Model" = None, prop_4: Optional[Dict[str, "_Model"]] = None,
                 prop_5: Optional[Union["_Model", List["_Model"]]] = None):
        super().__init__(locals())


@pytest.mark.parametrize("kwargs", [
    {"prop_0": 1}, {"prop_0": None}, {"prop_0": _Model(prop_0="x")},
    {"prop_0": "", "prop_1": 1},
    {"prop_0": "", "prop_2": None}, {"prop_0": "", "prop_2": 22.22},
    {"prop_0": "", "prop_3": 1}, {"prop_0": "", "prop_3": "s"}, {"prop_0": "", "prop_3": [_Model(prop_0="x")]},
    {"prop_0": "", "prop_4": "s"}, {"prop_0": "", "prop_4": {42: _Model(prop_0="x")}},
    {"prop_0": "", "prop_4": {"k": [_Model(prop_0="x")]}},
    {"prop_0": "", "prop_5": 1}, {"prop_0": "", "prop_5": {"k": "v"}},
])
def test_model_base_rejects_mistyped_fields(kwargs):
    with pytest.raises(TypeError):
        _Model(**kwargs)


def test_model_base_accepts_typed_fields():
    v = _Model(prop_0="v")
    assert _Model(prop_0="", prop_1=None).prop_1 is None
    assert [_Model(prop_0="", prop_2=x).prop_2 for x in ("s", 22, True)] == ["s", 22, True]
    assert _Model(prop_0="", prop_3=v).prop_3 is v
    assert _Model(prop_0="", prop_4={"k": v}).prop_4["k"] is v
    assert _Model(prop_0="", prop_5=[v]).prop_5[0] is v


@pytest.mark.parametrize("struct", [
    {"prop_0": "value 0"},
    {"prop_0": "", "prop1": "value 1"},
    {"prop_0": "", "prop 2": 22},
    {"prop_0": "", "@@": {"prop_0": "nested"}},
    {"prop_0": "", "prop_4": {"k": {"prop_0": "nested"}}},
    {"prop_0": "", "prop_5": [{"prop_0": "a"}, {"prop_0": "b", "prop 2": True}]},
])
def test_model_base_dict_round_trip_uses_serialized_names(struct):
    obj = _Model.from_dict(struct)
    assert obj.to_dict() == struct


def test_model_base_from_dict_rejects_non_dict():
    with pytest.raises((AttributeError, TypeError)):
        _Model.from_dict(None)


def test_component_spec_yaml_round_trip():
    text = ("name: Echo\ninputs:\n- {name: Msg, type: String, default: hi}\noutputs:\n- {name: Out}\n" + BUSYBOX +
            "    command: [sh, -c, 'echo \"$0\" > \"$1\"', {inputValue: Msg}, {outputPath: Out}]\n")
    spec = ComponentSpec.from_dict(load_yaml(text))
    assert ComponentSpec.from_dict(spec.to_dict()).to_dict() == spec.to_dict()
    assert spec.to_dict()["inputs"] == [{"name": "Msg", "type": "String", "default": "hi"}]
