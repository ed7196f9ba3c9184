"""CLI entry point (reference: `sdk/python/kfp/cli/cli.py:15-30`)."""
from __future__ import annotations

import click

from .._client import Client
from .run import run


@click.group()
@click.option("--endpoint", help="Endpoint of the pipelines API service ('local' or 'local://DIR' runs on this host).")
@click.option("--iap-client-id", help="Client ID for IAP protected endpoint.")
@click.option("-n", "--namespace", default="kubeflow", help="Kubernetes namespace to connect to the API.")
@click.pass_context
def cli(ctx, endpoint, iap_client_id, namespace):
    """Command line interface to the pipelines service."""
    ctx.obj["client"] = Client(endpoint, iap_client_id, namespace)
    ctx.obj["namespace"] = namespace


cli.add_command(run)


def main(argv=None):
    cli(args=argv, obj={}, auto_envvar_prefix="KFP")
