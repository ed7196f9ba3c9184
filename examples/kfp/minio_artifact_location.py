"""Pipeline-level Minio/S3 artifact repository (reference `kubeflow-pipelines/minio/minio.py:25-44`,
compiled by `minio/compile.sh` with `dsl-compile --py minio.py --output minio.tar.gz`): every output
artifact of every op is stored under `runs/{{workflow.uid}}/{{pod.name}}/<name>.tgz` in the bucket
on `minio-service.<namespace>:9000`, with credentials from the `mlpipeline-minio-artifact` secret.

    dsl-compile --py examples/kfp/minio_artifact_location.py --output minio.tar.gz"""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.kfp import dsl  # noqa: E402
from mifx.kfp.k8s import V1SecretKeySelector  # noqa: E402

SECRET = "mlpipeline-minio-artifact"


@dsl.pipeline(name="custom_artifact_location_pipeline",
              description="Store every op's artifacts in a Minio bucket configured once for the pipeline.")
def minio_artifacts(tag: str = "latest", namespace: str = "kubeflow", bucket: str = "mybucket"):
    dsl.get_pipeline_conf().set_artifact_location(dsl.ArtifactLocation.s3(
        bucket=bucket, endpoint=f"minio-service.{namespace}:9000", insecure=True,
        access_key_secret=V1SecretKeySelector(name=SECRET, key="accesskey"),
        secret_key_secret={"name": SECRET, "key": "secretkey"}))
    dsl.ContainerOp(name="foo", image=f"busybox:{tag}")


if __name__ == "__main__":
    from mifx.kfp import compiler

    compiler.Compiler().compile(minio_artifacts, (sys.argv[1] if len(sys.argv) > 1 else __file__ + ".tar.gz"))
