from __future__ import annotations

import os
import tempfile


def docker(line: str, cell: str):
    """%%docker <target-image> <staging-location>: build the Dockerfile in the cell with kaniko."""
    from ..compiler import build_docker_image

    if len(line.split()) != 2:
        raise ValueError("usage: %%docker [registry/image:tag] [gs://staging-bucket | /local/staging/dir]")
    if not cell.strip():
        raise ValueError("Please fill in a dockerfile content in the cell.")
    target, staging = line.split()
    with tempfile.NamedTemporaryFile(mode="wt", delete=False) as f:
        f.write(cell)
    try:
        build_docker_image(staging, target, f.name)
    finally:
        os.remove(f.name)


try:
    import IPython  # type: ignore

    if IPython.get_ipython() is not None:
        docker = IPython.core.magic.register_cell_magic(docker)
except ImportError:
    pass
