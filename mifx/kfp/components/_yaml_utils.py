"""Order-preserving YAML load/dump (reference: `sdk/python/kfp/components/_yaml_utils.py:17-56`)."""
from __future__ import annotations

from collections import OrderedDict

import yaml


class _OrderedLoader(yaml.SafeLoader):
    pass


def _construct_mapping(loader, node):
    loader.flatten_mapping(node)
    return OrderedDict(loader.construct_pairs(node))


_OrderedLoader.add_constructor(yaml.resolver.BaseResolver.DEFAULT_MAPPING_TAG, _construct_mapping)


class _OrderedDumper(yaml.SafeDumper):
    def ignore_aliases(self, data):
        return True


def _represent_ordered(dumper, data):
    return dumper.represent_mapping(yaml.resolver.BaseResolver.DEFAULT_MAPPING_TAG, data.items())


_OrderedDumper.add_representer(OrderedDict, _represent_ordered)


def _str_presenter(dumper, data):
    if "\n" in data:
        return dumper.represent_scalar("tag:yaml.org,2002:str", data, style="|")
    return dumper.represent_scalar("tag:yaml.org,2002:str", data)


_OrderedDumper.add_representer(str, _str_presenter)


def load_yaml(stream):
    return yaml.load(stream, Loader=_OrderedLoader)


def dump_yaml(data) -> str:
    return yaml.dump(data, Dumper=_OrderedDumper, default_flow_style=False, sort_keys=False)
