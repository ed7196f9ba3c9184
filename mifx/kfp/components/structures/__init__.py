"""Typed component-spec sub-structures (reference: `sdk/python/kfp/components/structures/`)."""
