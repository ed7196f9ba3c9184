"""Component registry over local directories and URL prefixes with digest / tag lookup.

Reference: `sdk/python/kfp/components/_component_store.py:10-93`."""
from __future__ import annotations

import os

from ._components import _create_task_factory_from_component_text
from ._structures import ComponentReference


class ComponentStore:
    def __init__(self, local_search_paths=None, url_search_prefixes=None):
        self.local_search_paths = local_search_paths or ["."]
        self.url_search_prefixes = url_search_prefixes or []
        self._component_file_name = "component.yaml"
        self._digests_subpath = "versions/sha256"
        self._tags_subpath = "versions/tags"

    def load_component_from_url(self, url: str):
        from ._components import load_component_from_url

        return load_component_from_url(url)

    def load_component_from_file(self, path: str):
        from ._components import load_component_from_file

        return load_component_from_file(path)

    def load_component(self, name: str, digest: str | None = None, tag: str | None = None):
        if not name:
            raise ValueError("name is required")
        if name.startswith("/") or name.endswith("/"):
            raise ValueError('Component name should not start or end with slash: "{}"'.format(name))
        if digest and tag:
            raise ValueError("Cannot specify both tag and digest")
        rel = name
        if digest:
            rel = os.path.join(name, self._digests_subpath, digest)
        elif tag:
            rel = os.path.join(name, self._tags_subpath, tag)
        tried = []
        for base in self.local_search_paths:
            p = os.path.join(base, rel, self._component_file_name)
            tried.append(p)
            if os.path.isfile(p):
                with open(p, "rb") as f:
                    return _create_task_factory_from_component_text(
                        f, p, ComponentReference(name=name, digest=digest, tag=tag))
        for prefix in self.url_search_prefixes:
            url = prefix + rel + "/" + self._component_file_name
            tried.append(url)
            try:
                import requests

                r = requests.get(url, timeout=30)
                if r.status_code == 200:
                    return _create_task_factory_from_component_text(
                        r.content, url, ComponentReference(name=name, digest=digest, tag=tag, url=url))
            except Exception:  # noqa: BLE001 - try the next location
                continue
        raise RuntimeError(f"Component {name} was not found. Tried the following locations:\n" + "\n".join(tried))


ComponentStore.default_store = ComponentStore(local_search_paths=["."])
