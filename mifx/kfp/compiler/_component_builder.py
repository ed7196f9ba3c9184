"""Container image builder for Python components (kaniko in-cluster, or local docker).

Reference: `sdk/python/kfp/compiler/_component_builder.py:27-551` — dependency pinning into a
requirements file, Dockerfile generation, build-context tarball, a kaniko Pod spec whose layout is
pinned by `tests/compiler/testdata/kaniko.basic.yaml`, an entrypoint wrapper around the user's
function source, and `build_python_component` / `build_docker_image`.

MI355X-first differences: the default base image is a ROCm PyTorch image and the generated
Dockerfile does not reinstall Python on top of it; the staging location may be a local directory
(or `file://`) as well as `gs://` (the latter requires `google-cloud-storage`); the kaniko pod is
submitted through `K8sHelper` (kubectl), so no python kubernetes client is needed."""
from __future__ import annotations

import inspect
import logging
import os
import re
import shutil
import tarfile
import tempfile
import textwrap
import uuid
from collections import OrderedDict
from pathlib import Path

from ._k8s_helper import K8sHelper

DEFAULT_BASE_IMAGE = "rocm/pytorch:latest"
KANIKO_IMAGE = "gcr.io/kaniko-project/executor:v0.5.0"


class StagingHelper:
    """Upload/download/remove of build contexts on gs:// or a local/file:// path."""

    @staticmethod
    def _local(path: str) -> str | None:
        if path.startswith("file://"):
            return path[len("file://"):]
        if "://" not in path:
            return path
        return None

    @staticmethod
    def _gcs_blob(gcs_path: str):
        try:
            from google.cloud import storage  # type: ignore
        except ImportError as e:  # pragma: no cover - optional dependency
            raise RuntimeError("gs:// staging requires google-cloud-storage") from e
        bucket, _, blob = gcs_path[len("gs://"):].partition("/")
        return storage.Client().get_bucket(bucket).blob(blob)

    @classmethod
    def upload(cls, local_path: str, remote: str) -> None:
        dst = cls._local(remote)
        if dst is not None:
            os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
            shutil.copyfile(local_path, dst)
        else:
            cls._gcs_blob(remote).upload_from_filename(local_path)

    @classmethod
    def download(cls, local_path: str, remote: str) -> None:
        src = cls._local(remote)
        if src is not None:
            shutil.copyfile(src, local_path)
        else:
            cls._gcs_blob(remote).download_to_filename(local_path)

    @classmethod
    def remove(cls, remote: str) -> None:
        p = cls._local(remote)
        if p is not None:
            if os.path.exists(p):
                os.remove(p)
        else:
            cls._gcs_blob(remote).delete()


GCSHelper = StagingHelper  # reference name


class VersionedDependency:
    """A python package with an exact version or a [min, max] range."""

    def __init__(self, name: str, version: str | None = None, min_version: str | None = None,
                 max_version: str | None = None):
        self._name = name
        if version is not None:
            self._min_version = self._max_version = version
        else:
            self._min_version, self._max_version = min_version, max_version

    @property
    def name(self):
        return self._name

    @property
    def min_version(self):
        return self._min_version

    @min_version.setter
    def min_version(self, v):
        self._min_version = v

    @property
    def max_version(self):
        return self._max_version

    @max_version.setter
    def max_version(self, v):
        self._max_version = v

    def has_min_version(self) -> bool:
        return self._min_version is not None

    def has_max_version(self) -> bool:
        return self._max_version is not None

    def has_versions(self) -> bool:
        return self.has_min_version() or self.has_max_version()


class DependencyHelper:
    """Ordered set of python package requirements -> requirements.txt."""

    def __init__(self):
        self._python_packages: "OrderedDict[str, VersionedDependency]" = OrderedDict()

    @property
    def python_packages(self):
        return self._python_packages

    def add_python_package(self, dependency: VersionedDependency, override: bool = True) -> None:
        if dependency.name in self._python_packages and not override:
            return
        self._python_packages[dependency.name] = dependency

    def requirement_lines(self):
        for name, dep in self._python_packages.items():
            cons = []
            if dep.has_min_version():
                cons.append(" >= " + dep.min_version)
            if dep.has_max_version():
                cons.append(" <= " + dep.max_version)
            yield name + ",".join(cons)

    def generate_pip_requirements(self, target_file: str) -> None:
        Path(target_file).write_text("".join(line + "\n" for line in self.requirement_lines()))


class DockerfileHelper:
    """Writes the Dockerfile (+ requirements) and wraps the build context into a .tar.gz."""

    REQUIREMENT_FILE = "requirements.txt"

    def __init__(self, arc_dockerfile_name: str):
        self._arc_dockerfile_name = arc_dockerfile_name
        self._ARC_REQUIREMENT_FILE = self.REQUIREMENT_FILE

    def _generate_pip_requirement(self, dependency, requirement_filepath: str) -> None:
        h = DependencyHelper()
        for d in dependency:
            h.add_python_package(d)
        h.generate_pip_requirements(requirement_filepath)

    def dockerfile_text(self, base_image: str, python_filepath: str, has_requirement_file: bool,
                        python_version: str = "python3") -> str:
        if python_version not in ("python2", "python3"):
            raise ValueError("python_version has to be either python2 or python3")
        py, pip = ("python3", "pip3") if python_version == "python3" else ("python", "pip")
        lines = ["FROM " + base_image]
        if not base_image.startswith("rocm/"):  # ROCm images already carry python + pip
            pkgs = "python3 python3-pip python3-setuptools" if py == "python3" else "python python-pip python-setuptools"
            lines.append("RUN apt-get update -y && apt-get install --no-install-recommends -y -q " + pkgs)
        if has_requirement_file:
            lines.append(f"ADD {self.REQUIREMENT_FILE} /ml/")
            lines.append(f"RUN {pip} install -r /ml/{self.REQUIREMENT_FILE}")
        lines.append(f"ADD {python_filepath} /ml/")
        lines.append(f'ENTRYPOINT ["{py}", "/ml/{python_filepath}"]')
        return "\n".join(lines)

    def _generate_dockerfile_with_py(self, target_file, base_image, python_filepath, has_requirement_file,
                                     python_version):
        Path(target_file).write_text(self.dockerfile_text(base_image, python_filepath, has_requirement_file,
                                                          python_version))

    @staticmethod
    def _wrap_files_in_tarball(tarball_path: str, files: dict) -> None:
        if not tarball_path.endswith(".tar.gz"):
            raise ValueError("the tarball path should end with .tar.gz")
        with tarfile.open(tarball_path, "w:gz") as tb:
            for arcname, path in files.items():
                tb.add(path, arcname=arcname)

    def prepare_docker_tarball_with_py(self, arc_python_filename, python_filepath, base_image, local_tarball_path,
                                       python_version="python3", dependency=None):
        if python_version not in ("python2", "python3"):
            raise ValueError("python_version has to be either python2 or python3")
        with tempfile.TemporaryDirectory() as d:
            files = OrderedDict()
            has_req = bool(dependency)
            if has_req:
                req = os.path.join(d, self.REQUIREMENT_FILE)
                self._generate_pip_requirement(dependency, req)
            dockerfile = os.path.join(d, self._arc_dockerfile_name)
            self._generate_dockerfile_with_py(dockerfile, base_image, arc_python_filename, has_req, python_version)
            files[self._arc_dockerfile_name] = dockerfile
            files[arc_python_filename] = python_filepath
            if has_req:
                files[self.REQUIREMENT_FILE] = req
            self._wrap_files_in_tarball(local_tarball_path, files)

    def prepare_docker_tarball(self, dockerfile_path, local_tarball_path):
        self._wrap_files_in_tarball(local_tarball_path, {self._arc_dockerfile_name: dockerfile_path})


class CodeGenerator:
    """Line-based code emitter with an indentation level."""

    def __init__(self, indentation: str = "\t"):
        self._indentation = indentation
        self._code: list = []
        self._level = 0

    def begin(self):
        self._code, self._level = [], 0

    def indent(self):
        self._level += 1

    def dedent(self):
        if self._level == 0:
            raise Exception("CodeGenerator dedent error")
        self._level -= 1

    def writeline(self, line: str):
        self._code.append(self._indentation * self._level + line)

    def end(self) -> str:
        return "\n".join(self._code) + "\n"


def kaniko_pod_spec(namespace: str, dockerfile: str, context: str, destination: str,
                    credentials_secret: str | None = "user-gcp-sa") -> dict:
    """Kaniko build Pod. With `credentials_secret` the secret is mounted at /secret/gcp-credentials and
    GOOGLE_APPLICATION_CREDENTIALS points into it (same layout as the reference's golden)."""
    container = {
        "name": "kaniko",
        "args": ["--cache=true", "--dockerfile=" + dockerfile, "--context=" + context,
                 "--destination=" + destination],
        "image": KANIKO_IMAGE,
    }
    spec = {"restartPolicy": "Never", "containers": [container], "serviceAccountName": "default"}
    if credentials_secret:
        container["env"] = [{"name": "GOOGLE_APPLICATION_CREDENTIALS",
                             "value": "/secret/gcp-credentials/user-gcp-sa.json"}]
        container["volumeMounts"] = [{"mountPath": "/secret/gcp-credentials", "name": "gcp-credentials"}]
        spec["volumes"] = [{"name": "gcp-credentials", "secret": {"secretName": credentials_secret}}]
    return {"apiVersion": "v1", "metadata": {"generateName": "kaniko-", "namespace": namespace}, "kind": "Pod",
            "spec": spec}


class ImageBuilder:
    """Builds an image from a python function or a Dockerfile, staging the context at `gcs_base`."""

    def __init__(self, gcs_base: str, target_image: str, k8s_helper: K8sHelper | None = None):
        self._arc_dockerfile_name = "dockerfile"
        self._arc_python_filename = "main.py"
        self._tarball_name = str(uuid.uuid4()) + ".tar.gz"
        self._gcs_base = gcs_base
        if gcs_base.startswith("gs://"):
            self._check_gcs_path(gcs_base)
        self._gcs_path = os.path.join(gcs_base, self._tarball_name)
        self._target_image = target_image
        self._k8s = k8s_helper

    @staticmethod
    def _check_gcs_path(gcs_path: str) -> bool:
        if not gcs_path.startswith("gs://"):
            raise ValueError("Error: {} should be a GCS path.".format(gcs_path))
        return True

    def _generate_kaniko_spec(self, namespace, arc_dockerfile_name, gcs_path, target_image):
        return kaniko_pod_spec(namespace, arc_dockerfile_name, gcs_path, target_image)

    def _generate_entrypoint(self, component_func, python_version: str = "python3") -> str:
        """User function source (decorators stripped) + a wrapper that converts argv to the annotated
        types and writes str(return value) to the trailing output-file argument."""
        if python_version not in ("python2", "python3"):
            raise ValueError("python_version has to be either python2 or python3")
        spec = inspect.getfullargspec(component_func)
        args, ann = spec.args, spec.annotations
        inputs = {k: v for k, v in ann.items() if k != "return"}
        if len(args) != len(inputs):
            raise Exception("Some input arguments do not contain annotations.")
        if "return" in ann and ann["return"] not in (int, float, str, bool):
            raise Exception("Output type not supported and supported types are [int, float, str, bool]")
        src = textwrap.dedent(inspect.getsource(component_func))  # nested functions are indented
        m = re.search(r"\n([ \t]+)[\w]+", src)
        cg = CodeGenerator(indentation=m.group(1) if m else "\t")
        wrapper = "wrapper_" + component_func.__name__
        cg.begin()
        cg.writeline("def " + wrapper + "(" + "".join(a + "," for a in args) + "_output_file):")
        cg.indent()
        cg.writeline("output = " + component_func.__name__ + "(" +
                     ",".join(f"{inputs[a].__name__}({a})" for a in args) + ")")
        cg.writeline("import os")
        cg.writeline("os.makedirs(os.path.dirname(_output_file))")
        cg.writeline('with open(_output_file, "w") as data:')
        cg.indent()
        cg.writeline("data.write(str(output))")
        wrapper_code = cg.end()
        cg.begin()
        cg.writeline("import argparse")
        cg.writeline('parser = argparse.ArgumentParser(description="Parsing arguments")')
        for a in args:
            cg.writeline(f'parser.add_argument("{a}", type={inputs[a].__name__})')
        cg.writeline('parser.add_argument("_output_file", type=str)')
        cg.writeline("args = vars(parser.parse_args())")
        cg.writeline("")
        cg.writeline('if __name__ == "__main__":')
        cg.indent()
        cg.writeline(wrapper + "(**args)")
        lines = src.split("\n")
        start = next((i for i, ln in enumerate(lines) if ln.startswith("def ")), 0)
        if python_version == "python2":
            lines[start] = "def " + component_func.__name__ + "(" + ", ".join(args) + "):"
        return "\n".join(lines[start:]) + "\n" + wrapper_code + "\n" + cg.end()

    def _build_image_from_tarball(self, local_tarball_path: str, namespace: str, timeout: int) -> None:
        StagingHelper.upload(local_tarball_path, self._gcs_path)
        spec = self._generate_kaniko_spec(namespace, self._arc_dockerfile_name, self._gcs_path, self._target_image)
        k8s = self._k8s or K8sHelper()
        try:
            ok = k8s.run_job(spec, timeout)
        finally:
            StagingHelper.remove(self._gcs_path)
        if not ok:
            raise RuntimeError("kaniko image build failed")

    def build_image_from_func(self, component_func, namespace, base_image, timeout, dependency,
                              python_version="python3"):
        with tempfile.TemporaryDirectory() as d:
            py = os.path.join(d, self._arc_python_filename)
            Path(py).write_text(self._generate_entrypoint(component_func, python_version))
            tb = os.path.join(d, self._tarball_name)
            DockerfileHelper(self._arc_dockerfile_name).prepare_docker_tarball_with_py(
                self._arc_python_filename, py, base_image, tb, python_version, dependency)
            self._build_image_from_tarball(tb, namespace, timeout)

    def build_image_from_dockerfile(self, dockerfile_path, timeout, namespace):
        with tempfile.TemporaryDirectory() as d:
            tb = os.path.join(d, self._tarball_name)
            DockerfileHelper(self._arc_dockerfile_name).prepare_docker_tarball(dockerfile_path, tb)
            self._build_image_from_tarball(tb, namespace, timeout)


def _generate_pythonop(component_func, target_image: str, target_component_file: str | None = None):
    from ..components._components import _create_task_factory_from_component_spec
    from ..components._python_op import _python_function_name_to_component_name
    from ..components._structures import (ComponentSpec, ContainerImplementation, ContainerSpec, InputSpec,
                                          InputValuePlaceholder, OutputPathPlaceholder, OutputSpec)
    from ..components._yaml_utils import dump_yaml

    name = getattr(component_func, "_component_human_name", None) or \
        _python_function_name_to_component_name(component_func.__name__)
    desc = getattr(component_func, "_component_description", None) or \
        (component_func.__doc__.strip() if component_func.__doc__ else None)
    in_names = inspect.getfullargspec(component_func).args
    spec = ComponentSpec(
        name=name, description=desc, inputs=[InputSpec(name=n, type="str") for n in in_names],
        outputs=[OutputSpec(name="output")],
        implementation=ContainerImplementation(container=ContainerSpec(
            image=target_image,
            args=[InputValuePlaceholder(n) for n in in_names] + [OutputPathPlaceholder("output")])))
    target_component_file = target_component_file or getattr(component_func, "_component_target_component_file", None)
    if target_component_file:
        Path(target_component_file).write_text(dump_yaml(spec.to_dict()))
    return _create_task_factory_from_component_spec(spec)


def build_python_component(component_func, target_image, base_image=None, dependency=(), staging_gcs_path=None,
                           build_image=True, timeout=600, namespace="kubeflow", target_component_file=None,
                           python_version="python3"):
    """Build an image for `component_func` (unless build_image=False) and return its task factory."""
    if component_func is None:
        raise ValueError("component_func must not be None")
    if target_image is None:
        raise ValueError("target_image must not be None")
    if python_version not in ("python2", "python3"):
        raise ValueError("python_version has to be either python2 or python3")
    if build_image:
        if staging_gcs_path is None:
            raise ValueError("staging_gcs_path must not be None")
        base_image = base_image or getattr(component_func, "_component_base_image", None) or DEFAULT_BASE_IMAGE
        logging.info("Build an image that is based on %s and push the image to %s", base_image, target_image)
        ImageBuilder(staging_gcs_path, target_image).build_image_from_func(
            component_func, namespace=namespace, base_image=base_image, timeout=timeout,
            python_version=python_version, dependency=list(dependency))
    return _generate_pythonop(component_func, target_image, target_component_file)


def build_docker_image(staging_gcs_path, target_image, dockerfile_path, timeout=600, namespace="kubeflow"):
    """Build `dockerfile_path` with kaniko and push it to `target_image`."""
    ImageBuilder(staging_gcs_path, target_image).build_image_from_dockerfile(dockerfile_path, timeout, namespace)
