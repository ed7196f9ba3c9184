"""`dsl-compile` CLI: compile the @dsl.pipeline function(s) of a .py file or a pip package.

Reference: `sdk/python/kfp/compiler/main.py:26-122` (flags --py/--package/--namespace/--function/
--output/--disable-type-check; a PipelineCollectorContext captures every decorated function).
Usage: ``python -m mifx.kfp.compiler.main --py pipeline.py --output pipeline.tar.gz``"""
from __future__ import annotations

import argparse
import importlib
import os
import shutil
import subprocess
import sys
import tempfile

from .. import dsl
from .compiler import Compiler


def parse_arguments(argv=None):
    ap = argparse.ArgumentParser(prog="dsl-compile")
    ap.add_argument("--py", type=str, help="local absolute path to a py file.")
    ap.add_argument("--package", type=str, help="local path to a pip installable python package file.")
    ap.add_argument("--function", type=str, help="The name of the function to compile if there are multiple.")
    ap.add_argument("--namespace", type=str, help="The namespace for the pipeline function")
    ap.add_argument("--output", type=str, required=True, help="local path to the output workflow yaml file.")
    ap.add_argument("--disable-type-check", action="store_true", help="disable the type check, default is enabled.")
    return ap.parse_args(argv)


def _compile_pipeline_function(funcs, function_name, output_path, type_check):
    if not funcs:
        raise ValueError("A function with @dsl.pipeline decorator is required in the py file.")
    if len(funcs) > 1 and not function_name:
        raise ValueError(f"There are multiple pipelines: {[f.__name__ for f in funcs]}. Please specify --function.")
    if function_name:
        fn = next((f for f in funcs if f.__name__ == function_name), None)
        if fn is None:
            raise ValueError(f'The function "{function_name}" does not exist. Did you forget @dsl.pipeline decoration?')
    else:
        fn = funcs[0]
    Compiler().compile(fn, output_path, type_check)


class PipelineCollectorContext:
    def __enter__(self):
        funcs = []

        def add(func):
            funcs.append(func)
            return func

        self.old = dsl._pipeline._pipeline_decorator_handler
        dsl._pipeline._pipeline_decorator_handler = add
        return funcs

    def __exit__(self, *args):
        dsl._pipeline._pipeline_decorator_handler = self.old


def _fresh_import(name: str):
    for k in [k for k in sys.modules if k == name or k.startswith(name + ".")]:
        del sys.modules[k]
    return importlib.import_module(name)


def compile_package(package_path, namespace, function_name, output_path, type_check):
    tmp = tempfile.mkdtemp()
    sys.path.insert(0, tmp)
    try:
        subprocess.check_call([sys.executable, "-m", "pip", "install", "--no-deps", "--no-index", package_path,
                               "-t", tmp])
        with PipelineCollectorContext() as funcs:
            _fresh_import(namespace)
        _compile_pipeline_function(funcs, function_name, output_path, type_check)
    finally:
        del sys.path[0]
        shutil.rmtree(tmp)


def compile_pyfile(pyfile, function_name, output_path, type_check):
    sys.path.insert(0, os.path.dirname(os.path.abspath(pyfile)))
    try:
        with PipelineCollectorContext() as funcs:
            _fresh_import(os.path.splitext(os.path.basename(pyfile))[0])
        _compile_pipeline_function(funcs, function_name, output_path, type_check)
    finally:
        del sys.path[0]


def main(argv=None):
    a = parse_arguments(argv)
    if (a.py is None) == (a.package is None):
        raise ValueError("Either --py or --package is needed but not both.")
    if a.py:
        compile_pyfile(a.py, a.function, a.output, not a.disable_type_check)
    else:
        if a.namespace is None:
            raise ValueError("--namespace is required for compiling packages.")
        compile_package(a.package, a.namespace, a.function, a.output, not a.disable_type_check)


if __name__ == "__main__":
    main()
