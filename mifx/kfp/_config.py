"""Global SDK configuration (reference: `sdk/python/kfp/_config.py:15`)."""
TYPE_CHECK = True
