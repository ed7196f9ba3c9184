"""Notebook server (Jupyter-role equivalent): mifx.notebook_server.server."""
