"""`run list|submit|get` (reference: `sdk/python/kfp/cli/run.py:24-102`)."""
from __future__ import annotations

import json
import shutil
import subprocess
import sys
import time

import click
from tabulate import tabulate


@click.group()
def run():
    """manage run resources"""


@run.command("list")
@click.option("-e", "--experiment-id", help="Parent experiment ID of listed runs.")
@click.option("--max-size", default=100, help="Max size of the listed runs.")
@click.pass_context
def list_runs(ctx, experiment_id, max_size):
    """list recent runs"""
    resp = ctx.obj["client"].list_runs(experiment_id=experiment_id, page_size=max_size, sort_by="created_at des")
    if resp and resp.runs:
        _print_runs(resp.runs)
    else:
        print("No runs found.")


@run.command()
@click.option("-e", "--experiment-name", required=True, help="Experiment name of the run.")
@click.option("-r", "--run-name", help="Name of the run.")
@click.option("-f", "--package-file", type=click.Path(exists=True, dir_okay=False),
              help="Path of the pipeline package file.")
@click.option("-p", "--pipeline-id", help="ID of the pipeline template.")
@click.option("-w", "--watch", is_flag=True, default=False, help="Watch the run status until it finishes.")
@click.argument("args", nargs=-1)
@click.pass_context
def submit(ctx, experiment_name, run_name, package_file, pipeline_id, watch, args):
    """submit a run"""
    client = ctx.obj["client"]
    run_name = run_name or experiment_name
    if not package_file and not pipeline_id:
        print("You must provide one of [package_file, pipeline_id].")
        sys.exit(1)
    arg_dict = dict(a.split("=", 1) for a in args)
    exp = client.create_experiment(experiment_name)
    r = client.run_pipeline(exp.id, run_name, package_file, arg_dict, pipeline_id)
    print("Run {} is submitted".format(r.id))
    _display_run(client, ctx.obj["namespace"], r.id, watch)


@run.command()
@click.option("-w", "--watch", is_flag=True, default=False, help="Watch the run status until it finishes.")
@click.argument("run-id")
@click.pass_context
def get(ctx, watch, run_id):
    """display the details of a run"""
    _display_run(ctx.obj["client"], ctx.obj["namespace"], run_id, watch)


_FINAL = ("Succeeded", "Skipped", "Failed", "Error")


def _display_run(client, namespace, run_id, watch):
    r = client.get_run(run_id).run
    _print_runs([r])
    if not watch:
        return
    if client.is_local:
        detail = client.wait_for_run_completion(run_id, timeout=24 * 3600)
        print("Run is finished with status {}.".format(detail.run.status))
        return
    wf_name = None
    while True:
        time.sleep(1)
        detail = client.get_run(run_id)
        if detail.pipeline_runtime and detail.pipeline_runtime.workflow_manifest:
            m = json.loads(detail.pipeline_runtime.workflow_manifest)
            if (m.get("metadata") or {}).get("name"):
                wf_name = m["metadata"]["name"]
                break
        if detail.run.status in _FINAL:
            print("Run is finished with status {}.".format(detail.run.status))
            return
    if wf_name and shutil.which("argo"):
        subprocess.run(["argo", "watch", wf_name, "-n", namespace])
    _print_runs([client.get_run(run_id).run])


def _print_runs(runs):
    data = [[r.id, r.name, r.status, r.created_at] for r in runs]
    print(tabulate(data, headers=["run id", "name", "status", "created at"], tablefmt="grid"))
