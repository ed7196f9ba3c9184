"""Pipelines exercising every compiler feature, written against `mifx.kfp`.

They describe the same workflows as the reference's compiler fixtures
(`sdk/python/tests/compiler/testdata/<name>.py`), so compiling `PIPELINES[name]` must produce a
Workflow equal to the reference's golden `<name>.yaml` (checked by tests/test_kfp_compiler.py when
the reference checkout is present; otherwise against digests recorded in golden_digests.json)."""
from __future__ import annotations

from mifx.kfp import dsl, gcp
from mifx.kfp.dsl import graph_component
from mifx.kfp.k8s import (V1EnvVar, V1ObjectMeta, V1ObjectReference, V1Secret, V1SecretKeySelector,
                          V1SecretVolumeSource, V1Volume, V1VolumeMount)

_WORD_CMD = ('python -c "from collections import Counter; '
             "words = Counter('%s'.split()); print(max(words, key=words.get))\" | tee /tmp/message.txt")
_FLIP_CMD = ("python -c \"import random; result = 'heads' if random.randint(0,1) == 0 else 'tails'; "
             "print(result)\" | tee /tmp/output")
_FAIL_CMD = "import random; import sys; exit_code = random.choice([%s]); print(exit_code); sys.exit(exit_code)"
_BASH = "library/bash:4.4.23"


def frequent_word_op(name, message):
    return dsl.ContainerOp(name=name, image="python:3.5-jessie", command=["sh", "-c"],
                           arguments=[_WORD_CMD % message], file_outputs={"word": "/tmp/message.txt"})


def save_message_op(name, message, output_path):
    return dsl.ContainerOp(name=name, image="google/cloud-sdk", command=["sh", "-c"],
                           arguments=["echo %s | tee /tmp/results.txt | gsutil cp /tmp/results.txt %s"
                                      % (message, output_path)])


def download_op(name, url):
    return dsl.ContainerOp(name=name, image="google/cloud-sdk", command=["sh", "-c"],
                           arguments=["gsutil cat %s | tee /tmp/results.txt" % url],
                           file_outputs={"downloaded": "/tmp/results.txt"})


def echo_op(name, msg):
    return dsl.ContainerOp(name=name, image="library/bash", command=["sh", "-c"], arguments=["echo %s" % msg])


def flip_op(name="Flip"):
    return dsl.ContainerOp(name=name, image="python:alpine3.6", command=["sh", "-c"], arguments=[_FLIP_CMD],
                           file_outputs={"output": "/tmp/output"})


def print_op(name, msg):
    return dsl.ContainerOp(name=name, image="alpine:3.6", command=["echo", msg])


def failing_op(exit_codes):
    return dsl.ContainerOp(name="random_failure", image="python:alpine3.6", command=["python", "-c"],
                           arguments=[_FAIL_CMD % exit_codes])


def bash_op(name, arguments=None, command=("sh", "-c"), pvolumes=None):
    return dsl.ContainerOp(name=name, image=_BASH, command=list(command), arguments=arguments, pvolumes=pvolumes)


PIPELINES = {}


def _register(name):
    def deco(fn):
        PIPELINES[name] = fn
        return fn
    return deco


@_register("basic")
@dsl.pipeline(name="Save Most Frequent", description="Get Most Frequent Word and Save to GCS")
def basic_pipeline(message: str, outputpath: str):
    exit_op = dsl.ContainerOp(name="exiting", image="python:3.5-jessie", command=["sh", "-c"],
                              arguments=["echo exit!"])
    with dsl.ExitHandler(exit_op):
        counter = frequent_word_op("get-Frequent", message)
        counter.set_memory_request("200M")
        saver = save_message_op("save", counter.output, outputpath)
        saver.set_cpu_limit("0.5")
        saver.set_gpu_limit("2")
        saver.add_node_selector_constraint("cloud.google.com/gke-accelerator", "nvidia-tesla-k80")
        saver.apply(gcp.use_tpu(tpu_cores=8, tpu_resource="v2", tf_version="1.12"))


@dsl.pipeline(name="Save Most Frequent", description="Get Most Frequent Word and Save to GCS")
def _save_most_frequent(message: dsl.PipelineParam, outputpath: dsl.PipelineParam):
    counter = frequent_word_op("get-Frequent", message)
    save_message_op("save", counter.output, outputpath)


@_register("compose")
@dsl.pipeline(name="Download and Save Most Frequent", description="Download and Get Most Frequent Word and Save to GCS")
def compose_pipeline(url: str, outputpath: str):
    downloader = download_op("download", url)
    _save_most_frequent(downloader.output, outputpath)


@_register("coin")
@dsl.pipeline(name="pipeline flip coin", description="shows how to use dsl.Condition.")
def coin_pipeline():
    flip = flip_op("flip")
    with dsl.Condition(flip.output == "heads"):
        flip2 = flip_op("flip-again")
        with dsl.Condition(flip2.output == "tails"):
            print_op("print1", flip2.output)
    with dsl.Condition(flip.output == "tails"):
        print_op("print2", flip2.output)


@_register("pipelineparams")
@dsl.pipeline(name="PipelineParams", description="A pipeline with multiple pipeline params.")
def pipelineparams_pipeline(tag: str = "latest", sleep_ms: int = 10):
    echo = dsl.Sidecar(name="echo", image="hashicorp/http-echo:%s" % tag, args=['-text="hello world"'])
    op1 = dsl.ContainerOp(name="download", image="busybox:%s" % tag, command=["sh", "-c"],
                          arguments=["sleep %s; wget localhost:5678 -O /tmp/results.txt" % sleep_ms],
                          sidecars=[echo], file_outputs={"downloaded": "/tmp/results.txt"})
    op2 = dsl.ContainerOp(name="echo", image="library/bash", command=["sh", "-c"],
                          arguments=["echo $MSG %s" % op1.output])
    op2.container.add_env_variable(V1EnvVar(name="MSG", value="pipelineParams: "))


@_register("sidecar")
@dsl.pipeline(name="Sidecar", description="A pipeline with sidecars.")
def sidecar_pipeline():
    echo = dsl.Sidecar(name="echo", image="hashicorp/http-echo", args=['-text="hello world"'])
    op1 = dsl.ContainerOp(name="download", image="busybox", command=["sh", "-c"],
                          arguments=["sleep 10; wget localhost:5678 -O /tmp/results.txt"], sidecars=[echo],
                          file_outputs={"downloaded": "/tmp/results.txt"})
    echo_op("echo", op1.output)


@_register("artifact_location")
@dsl.pipeline(name="foo", description="hello world")
def artifact_location_pipeline(tag: str, namespace: str = "kubeflow", bucket: str = "foobar"):
    minio = dsl.ArtifactLocation.s3(bucket=bucket, endpoint="minio-service.%s:9000" % namespace, insecure=True,
                                    access_key_secret={"name": "minio", "key": "accesskey"},
                                    secret_key_secret=V1SecretKeySelector(name="minio", key="secretkey"))
    s3 = dsl.ArtifactLocation.s3(bucket=bucket, endpoint="s3.amazonaws.com", region="ap-southeast-1", insecure=False)
    dsl.get_pipeline_conf().set_artifact_location(minio)
    dsl.ContainerOp(name="foo", image="busybox:%s" % tag)
    dsl.ContainerOp(name="foo", image="busybox:%s" % tag, artifact_location=s3)


@_register("default_value")
@dsl.pipeline(name="Default Value", description="A pipeline with parameter and default value.")
def default_value_pipeline(url="gs://ml-pipeline/shakespeare1.txt"):
    op1 = download_op("download", url)
    echo_op("echo", op1.output)


@_register("immediate_value")
@dsl.pipeline(name="Immediate Value", description="A pipeline with parameter values hard coded")
def immediate_value_pipeline():
    url = dsl.PipelineParam(name="url", value="gs://ml-pipeline/shakespeare1.txt")
    op1 = download_op("download", url)
    echo_op("echo", op1.output)


@_register("imagepullsecret")
@dsl.pipeline(name="Save Most Frequent", description="Get Most Frequent Word and Save to GCS")
def imagepullsecret_pipeline(message: str):
    frequent_word_op("get-Frequent", message)
    dsl.get_pipeline_conf().set_image_pull_secrets([V1ObjectReference(name="secretA")])


@_register("param_op_transform")
@dsl.pipeline(name="Parameters in Op transformation functions",
              description="Test that parameters used in Op transformation functions as pod labels "
                          "would be correcly identified and set as arguments in he generated yaml")
def param_op_transform_pipeline(param=dsl.PipelineParam(name="param")):
    dsl.get_pipeline_conf().op_transformers.append(lambda op: op.add_pod_label("param", param))
    dsl.ContainerOp(name="cop", image="image")


@_register("param_substitutions")
@dsl.pipeline(name="Param Substitutions",
              description="Test the same PipelineParam getting substituted in multiple places")
def param_substitutions_pipeline():
    vop = dsl.VolumeOp(name="create_volume", resource_name="data", size="1Gi")
    dsl.ContainerOp(name="cop", image="image", arguments=["--param", vop.output], pvolumes={"/mnt": vop.volume})


def _recursive_do_while():
    @graph_component
    def flip_component(flip_result):
        shown = print_op("Print", flip_result)
        flip = flip_op().after(shown)
        with dsl.Condition(flip.output == "heads"):
            flip_component(flip.output)

    @dsl.pipeline(name="pipeline flip coin", description="shows how to use graph_component.")
    def recursive():
        flip_a, flip_b = flip_op(), flip_op()
        loop = flip_component(flip_a.output)
        loop.after(flip_b)
        print_op("Print", "cool, it is over. %s" % flip_a.output).after(loop)

    return recursive


def _recursive_while():
    @graph_component
    def flip_component(flip_result):
        with dsl.Condition(flip_result == "heads"):
            shown = print_op("Print", flip_result)
            flip = flip_op().after(shown)
            flip_component(flip.output)

    @dsl.pipeline(name="pipeline flip coin", description="shows how to use dsl.Condition.")
    def flipcoin():
        flip_a, flip_b = flip_op(), flip_op()
        loop = flip_component(flip_a.output)
        loop.after(flip_b)
        print_op("Print", "cool, it is over. %s" % flip_a.output).after(loop)

    return flipcoin


PIPELINES["recursive_do_while"] = _recursive_do_while()
PIPELINES["recursive_while"] = _recursive_while()


@_register("resourceop_basic")
@dsl.pipeline(name="ResourceOp Basic", description="A Basic Example on ResourceOp Usage.")
def resourceop_basic(username, password):
    secret = V1Secret(api_version="v1", kind="Secret", metadata=V1ObjectMeta(generate_name="my-secret-"),
                      type="Opaque", data={"username": username, "password": password})
    rop = dsl.ResourceOp(name="create-my-secret", k8s_resource=secret,
                         attribute_outputs={"name": "{.metadata.name}"})
    vol = V1Volume(name="my-secret", secret=V1SecretVolumeSource(secret_name=rop.output))
    bash_op("cop", ["ls /etc/secret-volume"], pvolumes={"/etc/secret-volume": vol})


@_register("retry")
@dsl.pipeline(name="pipeline includes two steps which fail randomly.",
              description="shows how to use ContainerOp set_retry().")
def retry_pipeline():
    failing_op("0,1,2,3").set_retry(100)
    failing_op("0,1").set_retry(50)


@_register("timeout")
@dsl.pipeline(name="pipeline includes two steps which fail randomly.",
              description="shows how to use ContainerOp set_retry().")
def timeout_pipeline():
    failing_op("0,1,2,3").set_timeout(10)
    failing_op("0,1")
    dsl.get_pipeline_conf().set_timeout(50)


@_register("volume")
@dsl.pipeline(name="Volume", description="A pipeline with volume.")
def volume_pipeline():
    op1 = dsl.ContainerOp(name="download", image="google/cloud-sdk", command=["sh", "-c"],
                          arguments=["ls | tee /tmp/results.txt"], file_outputs={"downloaded": "/tmp/results.txt"}) \
        .add_volume(V1Volume(name="gcp-credentials", secret=V1SecretVolumeSource(secret_name="user-gcp-sa"))) \
        .add_volume_mount(V1VolumeMount(mount_path="/secret/gcp-credentials", name="gcp-credentials")) \
        .add_env_variable(V1EnvVar(name="GOOGLE_APPLICATION_CREDENTIALS",
                                   value="/secret/gcp-credentials/user-gcp-sa.json")) \
        .add_env_variable(V1EnvVar(name="Foo", value="bar"))
    echo_op("echo", op1.output)


@_register("volumeop_basic")
@dsl.pipeline(name="VolumeOp Basic", description="A Basic Example on VolumeOp Usage.")
def volumeop_basic(size):
    vop = dsl.VolumeOp(name="create_pvc", resource_name="my-pvc", modes=dsl.VOLUME_MODE_RWM, size=size)
    bash_op("cop", ["echo foo > /mnt/file1"], pvolumes={"/mnt": vop.volume})


@_register("volumeop_dag")
@dsl.pipeline(name="Volume Op DAG", description="The second example of the design doc.")
def volumeop_dag():
    vop = dsl.VolumeOp(name="create_pvc", resource_name="my-pvc", size="10Gi", modes=dsl.VOLUME_MODE_RWM)
    s1 = bash_op("step1", ["echo 1 | tee /mnt/file1"], pvolumes={"/mnt": vop.volume})
    s2 = bash_op("step2", ["echo 2 | tee /mnt2/file2"], pvolumes={"/mnt2": vop.volume})
    bash_op("step3", ["cat /mnt/file1 /mnt/file2"], pvolumes={"/mnt": vop.volume.after(s1, s2)})


@_register("volumeop_parallel")
@dsl.pipeline(name="VolumeOp Parallel", description="The first example of the design doc.")
def volumeop_parallel():
    vop = dsl.VolumeOp(name="create_pvc", resource_name="my-pvc", size="10Gi", modes=dsl.VOLUME_MODE_RWM)
    bash_op("step1", ["echo 1 | tee /mnt/file1"], pvolumes={"/mnt": vop.volume})
    bash_op("step2", ["echo 2 | tee /common/file2"], pvolumes={"/common": vop.volume})
    bash_op("step3", ["echo 3 | tee /mnt3/file3"], pvolumes={"/mnt3": vop.volume})


@_register("volumeop_sequential")
@dsl.pipeline(name="VolumeOp Sequential", description="The third example of the design doc.")
def volumeop_sequential():
    vop = dsl.VolumeOp(name="mypvc", resource_name="newpvc", size="10Gi", modes=dsl.VOLUME_MODE_RWM)
    s1 = bash_op("step1", ["echo 1|tee /data/file1"], pvolumes={"/data": vop.volume})
    s2 = bash_op("step2", ["cp /data/file1 /data/file2"], pvolumes={"/data": s1.pvolume})
    bash_op("step3", command=["cat", "/mnt/file1", "/mnt/file2"], pvolumes={"/mnt": s2.pvolume})


@_register("volume_snapshotop_sequential")
@dsl.pipeline(name="VolumeSnapshotOp Sequential", description="The fourth example of the design doc.")
def volume_snapshotop_sequential(url):
    vop = dsl.VolumeOp(name="create_volume", resource_name="vol1", size="1Gi", modes=dsl.VOLUME_MODE_RWM)
    s1 = dsl.ContainerOp(name="step1_ingest", image="google/cloud-sdk:216.0.0", command=["sh", "-c"],
                         arguments=["mkdir /data/step1 && gsutil cat %s | gzip -c >/data/step1/file1.gz" % url],
                         pvolumes={"/data": vop.volume})
    dsl.VolumeSnapshotOp(name="step1_snap", resource_name="step1_snap", volume=s1.pvolume)
    s2 = bash_op("step2_gunzip", ["mkdir /data/step2 && gunzip /data/step1/file1.gz -c >/data/step2/file1"],
                 pvolumes={"/data": s1.pvolume})
    dsl.VolumeSnapshotOp(name="step2_snap", resource_name="step2_snap", volume=s2.pvolume)
    s3 = bash_op("step3_copy", ["mkdir /data/step3 && cp -av /data/step2/file1 /data/step3/file3"],
                 pvolumes={"/data": s2.pvolume})
    dsl.VolumeSnapshotOp(name="step3_snap", resource_name="step3_snap", volume=s3.pvolume)
    bash_op("step4_output", command=["cat", "/data/step2/file1", "/data/step3/file3"], pvolumes={"/data": s3.pvolume})


@_register("volume_snapshotop_rokurl")
@dsl.pipeline(name="VolumeSnapshotOp RokURL", description="The fifth example of the design doc.")
def volume_snapshotop_rokurl(rok_url):
    vop1 = dsl.VolumeOp(name="create_volume_1", resource_name="vol1", size="1Gi",
                        annotations={"rok/origin": rok_url}, modes=dsl.VOLUME_MODE_RWM)
    s1 = bash_op("step1_concat", ["cat /data/file*| gzip -c >/data/full.gz"], pvolumes={"/data": vop1.volume})
    snap1 = dsl.VolumeSnapshotOp(name="create_snapshot_1", resource_name="snap1", volume=s1.pvolume)
    vop2 = dsl.VolumeOp(name="create_volume_2", resource_name="vol2", data_source=snap1.snapshot,
                        size=snap1.outputs["size"])
    s2 = bash_op("step2_gunzip", command=["gunzip", "-k", "/data/full.gz"], pvolumes={"/data": vop2.volume})
    snap2 = dsl.VolumeSnapshotOp(name="create_snapshot_2", resource_name="snap2", volume=s2.pvolume)
    vop3 = dsl.VolumeOp(name="create_volume_3", resource_name="vol3", data_source=snap2.snapshot,
                        size=snap2.outputs["size"])
    bash_op("step3_output", command=["cat", "/data/full"], pvolumes={"/data": vop3.volume})
