"""DSL object-level unit tests (no compiler, no backend).

Mirrors the reference's `sdk/python/tests/dsl/*` strategy ("the fixture is the
`with Pipeline('somename') as p:` context"): ops register into `p.ops`, groups nest into `p.groups`,
PipelineParams serialise/parse, resource/volume/snapshot ops derive their attribute outputs, and the
platform op-modifiers add the documented env vars. Behaviour pinned to the reference files cited per test.
"""
import inspect
import warnings

import pytest

from mifx.kfp import aws, azure, gcp, onprem
from mifx.kfp import dsl
from mifx.kfp.compiler._k8s_helper import K8sHelper
from mifx.kfp.dsl import (ArtifactLocation, ContainerOp, ExitHandler, OpsGroup, Pipeline, PipelineParam,
                          PipelineVolume, ResourceOp, Sidecar, VolumeOp, VolumeSnapshotOp, component, pipeline)
from mifx.kfp.dsl._metadata import ComponentMeta, ParameterMeta, PipelineMeta, TypeMeta, _extract_pipeline_metadata
from mifx.kfp.dsl._pipeline_param import _extract_pipelineparams, extract_pipelineparams_from_any
from mifx.kfp.dsl.types import GCSPath, InconsistentTypeException, Integer, _instance_to_dict, check_types
from mifx.kfp.k8s import (V1Container, V1EnvVar, V1ObjectMeta, V1PersistentVolumeClaim,
                          V1PersistentVolumeClaimVolumeSource, V1SecretKeySelector, V1TypedLocalObjectReference,
                          V1VolumeMount)


# ---------------------------------------------------------------- Pipeline context (_pipeline.py:177-229)

def test_pipeline_context_registers_ops_and_resets_default():
    assert Pipeline.get_default_pipeline() is None
    with Pipeline("ctx") as p:
        assert Pipeline.get_default_pipeline() is p
        ContainerOp(name="first", image="img")
        ContainerOp(name="second", image="img")
    assert Pipeline.get_default_pipeline() is None
    assert [p.ops[k].name for k in ("first", "second")] == ["first", "second"]


def test_duplicate_op_names_get_index_suffix():
    # _pipeline.py:203-204: the second 'step' becomes 'step 2' (space-delimited; the compiler's name
    # sanitiser turns it into 'step-2' in the workflow, golden recursive_while.yaml)
    with Pipeline("dups") as p:
        a = ContainerOp(name="step", image="img")
        b = ContainerOp(name="step", image="img")
        c = ContainerOp(name="step", image="img")
    assert (a.name, b.name, c.name) == ("step", "step 2", "step 3")
    assert set(p.ops) == {"step", "step 2", "step 3"}
    assert K8sHelper.sanitize_k8s_name(b.name) == "step-2"


def test_nested_pipeline_contexts_are_rejected():
    with pytest.raises(Exception):
        with Pipeline("outer"):
            with Pipeline("inner"):
                pass
    assert Pipeline.get_default_pipeline() is None


def test_pipeline_decorator_records_name_and_description():
    @pipeline(name="alpha", description="first")
    def f1():
        pass

    @pipeline(name="beta", description="second")
    def f2():
        pass

    assert (f1._pipeline_name, f1._pipeline_description) == ("alpha", "first")
    assert (f2._pipeline_name, f2._pipeline_description) == ("beta", "second")


def test_pipeline_metadata_from_annotations():
    @pipeline(name="meta", description="d")
    def f(a: {"Schema": {"file_type": "csv"}} = "good", b: Integer() = 12):  # noqa: F821
        pass

    meta = _extract_pipeline_metadata(f)
    want = PipelineMeta(name="meta", description="d")
    want.inputs.append(ParameterMeta(name="a", description="", default="good",
                                     param_type=TypeMeta(name="Schema", properties={"file_type": "csv"})))
    want.inputs.append(ParameterMeta(name="b", description="", default=12, param_type=TypeMeta(
        name="Integer", properties={"openapi_schema_validator": {"type": "integer"}})))
    assert meta == want


# ---------------------------------------------------------------- PipelineParam (_pipeline_param.py:146-241)

def test_pipeline_param_rejects_invalid_names():
    with pytest.raises(ValueError):
        PipelineParam(name="9lives")


@pytest.mark.parametrize("kwargs,text", [
    ({"name": "x", "op_name": "producer"}, "{{pipelineparam:op=producer;name=x;value=;type=;}}"),
    ({"name": "y"}, "{{pipelineparam:op=;name=y;value=;type=;}}"),
    ({"name": "z", "value": "v"}, "{{pipelineparam:op=;name=z;value=v;type=;}}"),
])
def test_pipeline_param_serialisation(kwargs, text):
    assert str(PipelineParam(**kwargs)) == text


def test_extract_params_from_strings_and_lists_dedups_in_order():
    typed = TypeMeta(name="custom", properties={"k": "v"})
    p1 = PipelineParam(name="p1", op_name="o1", param_type=typed)
    p2 = PipelineParam(name="p2", param_type=TypeMeta(name="bare"))
    p3 = PipelineParam(name="p3", value="three")
    joined = f"{p1} and {p2} and {p3}"
    assert _extract_pipelineparams(joined) == [p1, p2, p3]
    assert _extract_pipelineparams([f"{p1}-{p2}", f"{p2}/{p3}"]) == [p1, p2, p3]
    # the type survives the round trip through the serialised form
    got = _extract_pipelineparams(str(p1))[0]
    assert got.param_type == typed


def test_extract_params_from_k8s_objects():
    p1, p2, p3 = PipelineParam("a", op_name="o"), PipelineParam("b"), PipelineParam("c", value="3")
    cont = V1Container(name=p1, image=p2, env=[V1EnvVar(name="E", value=f"{p1} {p2} {p3}")])
    got = extract_pipelineparams_from_any(cont)
    assert sorted(got, key=str) == sorted([p1, p2, p3], key=str)


def test_pipeline_param_comparisons_build_condition_operators():
    p = PipelineParam("flip", op_name="coin")
    cond = p == "heads"
    assert (cond.operator, cond.operand1, cond.operand2) == ("==", p, "heads")
    assert (p > 3).operator == ">" and (p <= 3).operator == "<="


# ---------------------------------------------------------------- ContainerOp (_container_op.py:841-1078)

def test_container_op_inputs_outputs_sidecars_env():
    a, b = PipelineParam("a"), PipelineParam("b")
    op = (ContainerOp(name="op", image="img", arguments=[f"{a} x {b} y {a}"],
                      sidecars=[Sidecar(name="s0", image="i0")],
                      container_kwargs={"env": [V1EnvVar(name="E1", value="1")]},
                      file_outputs={"result": "/tmp/result"})
          .add_sidecar(Sidecar(name="s1", image="i1"))
          .add_sidecar(Sidecar(name="s2", image="i2")))
    assert sorted(x.name for x in op.inputs) == ["a", "b"]
    assert list(op.outputs) == ["result"] and op.outputs["result"].op_name == op.name
    assert op.output.name == "result"
    assert [s.name for s in op.sidecars] == ["s0", "s1", "s2"]
    assert [s.image for s in op.sidecars] == ["i0", "i1", "i2"]
    assert [e.name for e in op.container.env] == ["E1"]


def test_multiple_file_outputs_leave_output_unset():
    op = ContainerOp(name="op", image="img", file_outputs={"x": "/x", "y": "/y"})
    assert op.output is None and set(op.outputs) == {"x", "y"}


def test_after_records_dependency_names():
    o1 = ContainerOp(name="o1", image="img")
    o2 = ContainerOp(name="o2", image="img").after(o1)
    assert o2.dependent_names == [o1.name]


def test_retry_timeout_display_name_and_pod_metadata():
    op = (ContainerOp(name="o", image="img").set_retry(3).set_timeout(60).set_display_name("Pretty")
          .add_pod_annotation("a", "1").add_pod_label("l", "2").add_node_selector_constraint("gpu", "mi355x"))
    assert op.num_retries == 3 and op.timeout == 60 and op.display_name == "Pretty"
    assert op.pod_annotations == {"a": "1"} and op.pod_labels == {"l": "2"}
    assert op.node_selector == {"gpu": "mi355x"}


@pytest.mark.parametrize("vendor,key", [("nvidia", "nvidia.com/gpu"), ("amd", "amd.com/gpu")])
def test_gpu_limit_vendor_resource_name(vendor, key):
    op = ContainerOp(name="o", image="img")
    op.container.set_gpu_limit("2", vendor=vendor)
    assert op.container.resources.limits == {key: "2"}


def test_gpu_limit_rejects_unknown_vendor():
    with pytest.raises(ValueError):
        ContainerOp(name="o", image="img").container.set_gpu_limit("1", vendor="acme")


def test_resource_string_validation():
    c = ContainerOp(name="o", image="img").container
    c.set_memory_request("10Mi").set_cpu_limit("500m")
    assert c.resources.requests == {"memory": "10Mi"} and c.resources.limits == {"cpu": "500m"}
    with pytest.raises(ValueError):
        c.set_memory_limit("ten megs")
    with pytest.raises(ValueError):
        c.set_cpu_request("1.5.2")


def test_deprecated_container_proxies_warn():
    op = ContainerOp(name="o", image="img")
    calls = [
        lambda: setattr(op, "env_variables", [V1EnvVar(name="foo", value="bar")]),
        lambda: setattr(op, "image", "img2"),
        lambda: op.set_memory_request("10M"),
        lambda: op.set_memory_limit("10M"),
        lambda: op.set_cpu_request("100m"),
        lambda: op.set_cpu_limit("1"),
        lambda: op.set_gpu_limit("1"),
        lambda: op.add_env_variable(V1EnvVar(name="foo", value="bar")),
        lambda: op.add_volume_mount(V1VolumeMount(mount_path="/secret", name="s")),
    ]
    for call in calls:
        with pytest.warns(PendingDeprecationWarning):
            call()
    assert op.container.image == "img2"
    with pytest.warns(PendingDeprecationWarning):
        assert op.image == "img2"


# ---------------------------------------------------------------- Ops groups (_ops_group.py)

def test_nested_ops_groups_tree():
    with Pipeline("groups") as p:
        assert len(p.groups) == 1
        with OpsGroup(group_type="exit_handler"):
            ContainerOp(name="op1", image="img")
            with OpsGroup(group_type="branch"):
                ContainerOp(name="op2", image="img")
                ContainerOp(name="op3", image="img")
            with OpsGroup(group_type="loop"):
                ContainerOp(name="op4", image="img")
    (eh,) = p.groups[0].groups
    assert eh.type == "exit_handler" and [o.name for o in eh.ops] == ["op1"]
    branch, loop = eh.groups
    assert not branch.groups and sorted(o.name for o in branch.ops) == ["op2", "op3"]
    assert not loop.groups and [o.name for o in loop.ops] == ["op4"]


def test_graph_group_recursion_reference():
    with Pipeline("rec"):
        g1 = dsl.Graph("hello")
        g1.__enter__()
        assert not g1.recursive_ref and g1.name == "graph-hello-1"
        g2 = dsl.Graph("hello")  # same name while g1 is still open: a recursive call
        g2.__enter__()
        assert g2.recursive_ref is g1


def test_graph_group_name_prefix_is_not_recursion():
    with Pipeline("rec"):
        g1 = dsl.Graph("foo_bar")
        g1.__enter__()
        assert g1.name == "graph-foo-bar-1"
        g2 = dsl.Graph("foo")
        g2.__enter__()
        assert not g2.recursive_ref


def test_exit_handler_group():
    with Pipeline("eh") as p:
        cleanup = ContainerOp(name="cleanup", image="img")
        with ExitHandler(exit_op=cleanup):
            ContainerOp(name="work", image="img")
    eh = p.groups[0].groups[0]
    assert eh.type == "exit_handler" and eh.exit_op.name == "cleanup"
    assert [o.name for o in eh.ops] == ["work"]


def test_exit_op_with_dependencies_is_rejected():
    with pytest.raises(ValueError):
        with Pipeline("eh"):
            first = ContainerOp(name="first", image="img")
            cleanup = ContainerOp(name="cleanup", image="img").after(first)
            with ExitHandler(exit_op=cleanup):
                pass


def test_condition_group_records_operator():
    with Pipeline("cond") as p:
        flip = ContainerOp(name="flip", image="img", file_outputs={"output": "/out"})
        with dsl.Condition(flip.output == "heads"):
            ContainerOp(name="heads", image="img")
    cond = p.groups[0].groups[0]
    assert cond.type == "condition" and cond.condition.operand2 == "heads"
    assert [o.name for o in cond.ops] == ["heads"]


# ---------------------------------------------------------------- Resource / volume ops (_resource_op.py etc.)

def test_resource_op_attribute_outputs():
    with Pipeline("res"):
        cond = PipelineParam("cond")
        pvc = V1PersistentVolumeClaim(api_version="v1", kind="PersistentVolumeClaim",
                                      metadata=V1ObjectMeta(name="my-resource"))
        res = ResourceOp(name="resource", k8s_resource=pvc, success_condition=cond,
                         attribute_outputs={"test": "attr"})
    assert [x.name for x in res.inputs] == ["cond"]
    assert res.resource.action == "create" and res.resource.success_condition == PipelineParam("cond")
    assert res.resource.failure_condition is None and res.resource.manifest is None
    assert res.attribute_outputs == {"manifest": "{}", "name": "{.metadata.name}", "test": "attr"}
    assert res.outputs == {k: PipelineParam(name=k, op_name=res.name) for k in ("manifest", "name", "test")}
    assert res.output == PipelineParam(name="test", op_name=res.name)
    assert res.dependent_names == []


def test_volume_op_outputs_and_volume():
    with Pipeline("vol"):
        rn, sz = PipelineParam("rn"), PipelineParam("sz")
        vol = VolumeOp(name="myvol_creation", resource_name=rn, size=sz, annotations={"k": "v"})
    assert sorted(x.name for x in vol.inputs) == ["rn", "sz"]
    assert vol.k8s_resource.metadata.name == "{{workflow.name}}-%s" % PipelineParam("rn")
    assert vol.attribute_outputs == {"manifest": "{}", "name": "{.metadata.name}",
                                     "size": "{.status.capacity.storage}"}
    assert vol.output == PipelineParam(name="name", op_name=vol.name)
    assert vol.dependent_names == []
    assert vol.volume == PipelineVolume(
        name="myvol-creation",
        persistent_volume_claim=V1PersistentVolumeClaimVolumeSource(
            claim_name=PipelineParam(name="name", op_name=vol.name)))


def test_volume_op_validation():
    # _volume_op.py:73-99: size required and a valid memory string (unless a PipelineParam), k8s_resource
    # exclusive with the other arguments and a PVC, data_source a name / param / typed reference
    with Pipeline("vol"):
        with pytest.raises(ValueError):
            VolumeOp(name="v", resource_name="r")
        with pytest.raises(ValueError):
            VolumeOp(name="v", resource_name="r", size="ten gigs")
        VolumeOp(name="v", resource_name="r", size=PipelineParam("sz"))
        with pytest.raises(ValueError):
            VolumeOp(name="v", resource_name="r", size="1Gi",
                     k8s_resource=V1PersistentVolumeClaim(metadata=V1ObjectMeta(name="x")))
        with pytest.raises(ValueError):
            VolumeOp(name="v", k8s_resource={"kind": "PersistentVolumeClaim"})
        with pytest.raises(ValueError):
            VolumeOp(name="v", resource_name="r", size="1Gi", data_source=42)
        seeded = VolumeOp(name="v", resource_name="r", size="1Gi", data_source="snap")
    assert seeded.k8s_resource.spec.data_source == V1TypedLocalObjectReference(
        api_group="snapshot.storage.k8s.io", kind="VolumeSnapshot", name="snap")


def test_volume_snapshot_op_outputs():
    with Pipeline("snap"):
        p1, p2 = PipelineParam("p1"), PipelineParam("p2")
        vol = VolumeOp(name="myvol_creation", resource_name="myvol", size="1Gi")
        s1 = VolumeSnapshotOp(name="mysnap_creation", resource_name=p1, volume=vol.volume)
        s2 = VolumeSnapshotOp(name="mysnap_creation", resource_name="mysnap", pvc=p2,
                              attribute_outputs={"size": "test"})
    assert sorted(x.name for x in s1.inputs) == ["name", "p1"]
    assert [x.name for x in s2.inputs] == ["p2"]
    assert s1.attribute_outputs == {"manifest": "{}", "name": "{.metadata.name}", "size": "{.status.restoreSize}"}
    assert s2.attribute_outputs == {"manifest": "{}", "name": "{.metadata.name}", "size": "test"}
    assert s1.output == PipelineParam(name="name", op_name=s1.name)
    assert s2.output == PipelineParam(name="size", op_name=s2.name)
    assert s1.dependent_names == [] and s2.dependent_names == []
    assert s1.snapshot == V1TypedLocalObjectReference(api_group="snapshot.storage.k8s.io", kind="VolumeSnapshot",
                                                      name=PipelineParam(name="name", op_name=s1.name))


def test_pipeline_volume_carries_dependencies():
    with Pipeline("pv"):
        vol = VolumeOp(name="myvol_creation", resource_name="myvol", size="1Gi")
        op1 = ContainerOp(name="op1", image="img", pvolumes={"/mnt": vol.volume})
        op2 = ContainerOp(name="op2", image="img", pvolumes={"/data": op1.pvolume})
    assert vol.volume.dependent_names == []
    assert op1.pvolume.dependent_names == [op1.name]
    assert op2.dependent_names == [op1.name]
    assert [m.mount_path for m in op2.container.volume_mounts] == ["/data"]


def test_pipeline_volume_after_accumulates():
    with Pipeline("pv"):
        o1 = ContainerOp(name="o1", image="img")
        o2 = ContainerOp(name="o2", image="img").after(o1)
        o3 = ContainerOp(name="o3", image="img")
        v1 = PipelineVolume(name="pipeline-volume")
        v2 = v1.after(o1)
        v3 = v2.after(o2)
        v4 = v3.after(o1, o2)
        v5 = v4.after(o3)
    assert v1.dependent_names == [] and v2.dependent_names == ["o1"] and v3.dependent_names == ["o2"]
    assert sorted(v4.dependent_names) == ["o1", "o2"]
    assert sorted(v5.dependent_names) == ["o1", "o2", "o3"]


# ---------------------------------------------------------------- Artifact location (_artifact_location.py)

def _s3_location():
    return ArtifactLocation.s3(bucket="foo", endpoint="s3.amazonaws.com", insecure=False, region="ap-southeast-1",
                               access_key_secret={"name": "s3-secret", "key": "accesskey"},
                               secret_key_secret=V1SecretKeySelector(name="s3-secret", key="secretkey"))


def test_artifact_location_s3_fields():
    loc = _s3_location()
    assert (loc.s3.bucket, loc.s3.endpoint, loc.s3.insecure, loc.s3.region) == (
        "foo", "s3.amazonaws.com", False, "ap-southeast-1")
    assert (loc.s3.access_key_secret.name, loc.s3.access_key_secret.key) == ("s3-secret", "accesskey")
    assert (loc.s3.secret_key_secret.name, loc.s3.secret_key_secret.key) == ("s3-secret", "secretkey")


@pytest.mark.parametrize("as_dict", [False, True])
def test_create_artifact_for_s3(as_dict):
    loc = _s3_location()
    if as_dict:  # the compiler hands the location over as plain JSON
        loc = K8sHelper.convert_k8s_obj_to_json(loc)
    art = ArtifactLocation.create_artifact_for_s3(loc, name="foo", path="path/to", key="key")
    assert (art.name, art.path) == ("foo", "path/to")
    assert (art.s3.endpoint, art.s3.bucket, art.s3.key) == ("s3.amazonaws.com", "foo", "key")
    assert art.s3.access_key_secret.key == "accesskey" and art.s3.secret_key_secret.key == "secretkey"


def test_create_artifact_for_s3_without_location():
    art = ArtifactLocation.create_artifact_for_s3(None, name="foo", path="path/to", key="key")
    assert (art.name, art.path) == ("foo", "path/to")


# ---------------------------------------------------------------- types + metadata (types.py, _metadata.py)

def test_type_instance_to_dict():
    assert _instance_to_dict(GCSPath()) == {
        "GCSPath": {"openapi_schema_validator": {"type": "string", "pattern": "^gs://.*$"}}}


def test_check_types_is_structural_subset():
    csv = {"ArtifactA": {"path_type": "file", "file_type": "csv"}}
    assert check_types(csv, {"ArtifactA": {"path_type": "file", "file_type": "csv"}})
    assert not check_types(csv, {"ArtifactA": {"path_type": "file", "file_type": "tsv"}})
    full = {"A": {"X": "value1", "Y": "value2"}}
    assert not check_types(full, {"B": {"X": "value1", "Y": "value2"}})
    assert not check_types(full, {"A": {"X": "value1"}})
    assert check_types({"A": {"X": "value1"}}, full)
    assert not check_types(full, {"A": {"X": "value1", "Y": "value3"}})


def test_type_meta_deserialize_and_eq():
    assert TypeMeta.deserialize({"GCSPath": {"bucket_type": "directory"}}) == TypeMeta(
        name="GCSPath", properties={"bucket_type": "directory"})
    assert TypeMeta.deserialize("GCSPath") == TypeMeta(name="GCSPath")
    a = TypeMeta(name="GCSPath", properties={"file_type": "csv"})
    assert a == TypeMeta(name="GCSPath", properties={"file_type": "csv"})
    assert a != TypeMeta(name="GCSPath", properties={"file_type": "tsv"})
    assert a != TypeMeta(name="GCSPatha", properties={"file_type": "csv"})


def test_component_meta_to_dict():
    meta = ComponentMeta(name="c", description="desc", inputs=[
        ParameterMeta(name="i1", description="d1", default="x",
                      param_type=TypeMeta(name="GCSPath", properties={"file_type": "csv"})),
        ParameterMeta(name="i2", description="d2", default="y", param_type=TypeMeta(name="Integer")),
    ], outputs=[ParameterMeta(name="o1", description="d3", param_type=TypeMeta(name="Schema"))])
    assert meta.to_dict() == {
        "name": "c", "description": "desc",
        "inputs": [{"name": "i1", "description": "d1", "type": {"GCSPath": {"file_type": "csv"}}, "default": "x"},
                   {"name": "i2", "description": "d2", "type": "Integer", "default": "y"}],
        "outputs": [{"name": "o1", "description": "d3", "type": "Schema", "default": None}],
    }


# ---------------------------------------------------------------- @component type checking (_component.py:57-92)

class _MetaSink:
    def _set_metadata(self, m):
        self.meta = m


def test_component_decorator_attaches_metadata():
    @component
    def comp(a: {"ArtifactA": {"file_type": "csv"}}, b: Integer() = 12) -> {"model": Integer()}:  # noqa: F821
        return _MetaSink()

    got = comp(1, 2).meta
    want = ComponentMeta(name="comp", description="")
    want.inputs.append(ParameterMeta(name="a", description="",
                                     param_type=TypeMeta(name="ArtifactA", properties={"file_type": "csv"})))
    want.inputs.append(ParameterMeta(name="b", description="", default=12, param_type=TypeMeta(
        name="Integer", properties={"openapi_schema_validator": {"type": "integer"}})))
    want.outputs.append(ParameterMeta(name="model", description="", param_type=TypeMeta(
        name="Integer", properties={"openapi_schema_validator": {"type": "integer"}})))
    assert got == want


def _producer(out_type):
    @component
    def producer(n: Integer()) -> {"out": out_type}:  # noqa: F821
        return ContainerOp(name="producer", image="img", arguments=["--n", n], file_outputs={"out": "/out"})

    return producer


def _consumer(in_type):
    @component
    def consumer(x: in_type):  # noqa: F821
        return ContainerOp(name="consumer", image="img", arguments=["--x", x])

    return consumer


@pytest.mark.parametrize("out_type,in_type,ok", [
    (GCSPath(), GCSPath(), True),
    ("GCSPath", GCSPath(), True),             # bare name vs typed instance: the names agree
    ({"Art": {"p": "file", "f": "csv"}}, {"Art": {"p": "file", "f": "csv"}}, True),
    ({"Art": {"p": "file", "f": "tsv"}}, {"Art": {"p": "file", "f": "csv"}}, False),  # property value
    ({"ArtA": {"p": "file"}}, {"ArtB": {"p": "file"}}, False),                          # type name
    ("Integer", {"customized": {}}, False),
])
def test_component_type_check_between_ops(out_type, in_type, ok):
    import mifx.kfp as kfp_mod

    prev = kfp_mod.TYPE_CHECK
    kfp_mod.TYPE_CHECK = True
    try:
        with Pipeline("tc"):
            a = _producer(out_type)(12)
            if ok:
                _consumer(in_type)(a.outputs["out"])
            else:
                with pytest.raises(InconsistentTypeException):
                    _consumer(in_type)(a.outputs["out"])
        # with type checking off the same wiring is accepted
        kfp_mod.TYPE_CHECK = False
        with Pipeline("tc"):
            _consumer(in_type)(_producer(out_type)(12).outputs["out"])
    finally:
        kfp_mod.TYPE_CHECK = prev


# ---------------------------------------------------------------- platform op-modifiers (aws.py, azure.py, gcp.py)

def test_aws_secret_defaults_and_env():
    spec = inspect.getfullargspec(aws.use_aws_secret)
    assert spec.defaults == ("aws-secret", "AWS_ACCESS_KEY_ID", "AWS_SECRET_ACCESS_KEY")
    op = ContainerOp(name="o", image="img").apply(aws.use_aws_secret("mysecret", "kid", "sak"))
    env = op.container.env
    assert [(e.name, e.value_from.secret_key_ref.name, e.value_from.secret_key_ref.key) for e in env] == [
        ("AWS_ACCESS_KEY_ID", "mysecret", "kid"), ("AWS_SECRET_ACCESS_KEY", "mysecret", "sak")]


def test_azure_secret_defaults_and_env():
    assert inspect.getfullargspec(azure.use_azure_secret).defaults == ("azcreds",)
    op = ContainerOp(name="o", image="img").apply(azure.use_azure_secret("foo"))
    names = ["AZ_SUBSCRIPTION_ID", "AZ_TENANT_ID", "AZ_CLIENT_ID", "AZ_CLIENT_SECRET"]
    assert [e.name for e in op.container.env] == names
    assert all(e.value_from.secret_key_ref.name == "foo" and e.value_from.secret_key_ref.key == e.name
               for e in op.container.env)


def test_gcp_secret_mounts_volume_and_env():
    op = ContainerOp(name="o", image="img").apply(gcp.use_gcp_secret("user-gcp-sa"))
    assert any(v.name == "gcp-credentials-user-gcp-sa" for v in op.volumes)
    assert any(e.name == "GOOGLE_APPLICATION_CREDENTIALS" for e in op.container.env)


def test_onprem_mount_pvc():
    op = ContainerOp(name="o", image="img").apply(onprem.mount_pvc("users-pvc", "local-storage", "/mnt"))
    assert op.volumes[0].persistent_volume_claim.claim_name == "users-pvc"
    assert [(m.name, m.mount_path) for m in op.container.volume_mounts] == [("local-storage", "/mnt")]


# ---------------------------------------------------------------- k8s helper (_k8s_helper.py:125-183)

def test_k8s_helper_sanitize_and_convert():
    assert K8sHelper.sanitize_k8s_name("My__Op  Name!!") == "my-op-name"
    p = PipelineParam("size", op_name="make-vol")
    got = K8sHelper.convert_k8s_obj_to_json({"env": [V1EnvVar(name="E", value=p)], "n": 3, "t": (1, "a")})
    assert got == {"env": [{"name": "E", "value": "{{inputs.parameters.make-vol-size}}"}], "n": 3, "t": (1, "a")}


def test_no_warnings_on_plain_container_api():
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        op = ContainerOp(name="o", image="img")
        op.container.set_memory_limit("1Gi").add_env_variable(V1EnvVar(name="A", value="1"))
