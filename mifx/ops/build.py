"""In-tree native build for mifx (gfx950 HIP kernels + host C++ runtime pieces).

Every ``csrc/*.hip`` file becomes ``mifx/ops/lib/libmifx_<stem>.so`` (hipcc, gfx950 only) and
every ``csrc/*.cpp`` file becomes a host-only ``libmifx_<stem>.so`` (g++). The libraries expose
plain C ABIs that :mod:`mifx.ops._lib` binds with ctypes, so building needs no torch headers
and the ``.so`` files travel with the repository snapshot to the GPU box.

Usage: ``python -m mifx.ops.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import threading
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
LIBDIR = Path(__file__).resolve().parent / "lib"
ARCH = "gfx950"

HIP_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-shared",
    "-fPIC",
    "-std=c++17",
    "-Wno-unused-result",
    "-Wno-unused-value",
]
CXX_FLAGS = ["-O3", "-shared", "-fPIC", "-std=c++17", "-pthread", "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (expected /opt/rocm/bin/hipcc)")


def _file_flags(src: Path) -> list[str]:
    """Per-file extra flags from a `// MIFX_HIPCC_FLAGS: ...` line in the source."""
    for line in src.read_text().splitlines()[:80]:
        if line.startswith("// MIFX_HIPCC_FLAGS:"):
            return line.split(":", 1)[1].split()
    return []


def source_hash(src: Path) -> str:
    """sha256 (16 hex) of what a library is built from: its source, every csrc header, the compiler flags."""
    import hashlib

    h = hashlib.sha256()
    flags = (HIP_FLAGS + _file_flags(src)) if src.suffix == ".hip" else CXX_FLAGS
    h.update(" ".join(flags).encode())
    # the source and everything it #includes by quoted name, transitively (csrc/wd_chain64.hip builds
    # csrc/wd_chain.hip with another tile size; headers such as feed.h): a header edit rebuilds only its users
    for d in _quoted_includes(src):
        if d.name != HASH_HEADER.name:
            h.update(d.name.encode())
            h.update(d.read_bytes())
    return h.hexdigest()[:16]


def _quoted_includes(src: Path) -> list[Path]:
    seen: dict[Path, None] = {}
    todo = [src]
    while todo:
        f = todo.pop()
        if f in seen or not f.exists():
            continue
        seen[f] = None
        for ln in f.read_text().splitlines():
            t = ln.strip()
            if t.startswith('#include "'):
                name = t.split('"')[1]
                for base in (f.parent, CSRC, CSRC / "include"):
                    if (base / name).exists():
                        todo.append((base / name).resolve())
                        break
    return sorted(seen, key=lambda p: (p != src.resolve(), str(p)))


# force-included into every translation unit: the library reports the source hash it was built from, and
# mifx.ops._lib.load refuses a library whose hash does not match the sources next to it (no stale binaries)
HASH_HEADER = CSRC / "mifx_srchash.h"


def _needs_build(src: Path, out: Path) -> bool:
    if not out.exists():
        return True
    return embedded_hash(out) != source_hash(src)


def embedded_hash(lib: Path) -> str | None:
    """The hash string compiled into a library (read from the file, without loading it)."""
    data = lib.read_bytes()
    i = data.find(b"MIFX_SRC_HASH=")
    return data[i + 14:i + 30].decode(errors="replace") if i >= 0 else None


def _build_one(src: Path, force: bool) -> tuple[str, str]:
    out = LIBDIR / f"libmifx_{src.stem}.so"
    if not force and not _needs_build(src, out):
        return src.name, "up-to-date"
    tmp = out.with_suffix(f".so.tmp.{os.getpid()}.{threading.get_ident()}")
    hd = ["-include", str(HASH_HEADER), f"-DMIFX_SRC_HASH_VALUE=\"{source_hash(src)}\""]
    if src.suffix == ".hip":
        cmd = [hipcc()] + HIP_FLAGS + _file_flags(src) + hd + ["-I", str(CSRC), str(src), "-o", str(tmp)]
    else:
        cmd = [os.environ.get("CXX", "g++")] + CXX_FLAGS + hd + ["-I", str(CSRC), str(src), "-o", str(tmp)]
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        tmp.unlink(missing_ok=True)
        raise RuntimeError(f"build of {src.name} failed:\n{' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    tmp.replace(out)  # atomic: a concurrent loader sees the old or the new library, never a partial one
    return src.name, "built"


class build_lock:
    """Exclusive fcntl lock on LIBDIR/.build.lock: the N ranks of a data-parallel job that all find the libraries
    stale build them once (the first holder builds; the others wait, then find every library up to date)."""

    def __enter__(self):
        import fcntl

        LIBDIR.mkdir(parents=True, exist_ok=True)
        self._f = open(LIBDIR / ".build.lock", "w")
        fcntl.flock(self._f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *exc):
        import fcntl

        fcntl.flock(self._f, fcntl.LOCK_UN)
        self._f.close()


def build_all(force: bool = False, jobs: int | None = None, verbose: bool = True) -> list[Path]:
    srcs = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.cpp"))
    jobs = jobs or min(8, max(1, len(srcs)))
    with build_lock():  # staleness is re-checked per library under the lock (_build_one -> _needs_build)
        with cf.ThreadPoolExecutor(jobs) as ex:
            for name, status in ex.map(lambda s: _build_one(s, force), srcs):
                if verbose:
                    print(f"[mifx.build] {name}: {status}", file=sys.stderr)
    return [LIBDIR / f"libmifx_{s.stem}.so" for s in srcs]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    build_all(force=a.force, jobs=a.jobs)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
