"""Notebook helpers: the `%%docker` cell magic (reference: `sdk/python/kfp/notebook/_magic.py:15-44`)."""
from . import _magic  # noqa: F401
