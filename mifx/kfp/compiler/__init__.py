"""DSL -> Argo workflow compiler (+ component image builder)."""
from .compiler import Compiler, dump_yaml, read_package, write_package  # noqa: F401
from ._component_builder import build_docker_image, build_python_component  # noqa: F401
