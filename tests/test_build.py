"""Native build hygiene: every in-tree library carries the hash of the sources + flags it was built from, and the
loader refuses a library whose hash does not match the sources next to it (no stale binaries)."""
import pytest

from mifx.ops import _lib, build


def test_every_library_embeds_its_source_hash():
    srcs = sorted(build.CSRC.glob("*.hip")) + sorted(build.CSRC.glob("*.cpp"))
    assert len(srcs) >= 18
    for s in srcs:
        lib = build.LIBDIR / f"libmifx_{s.stem}.so"
        assert lib.exists(), lib
        assert build.embedded_hash(lib) == build.source_hash(s), s.name


def test_loader_refuses_a_stale_library(monkeypatch):
    monkeypatch.setenv("MIFX_AUTOBUILD", "0")
    monkeypatch.setattr(build, "source_hash", lambda src: "0000000000000000")
    with pytest.raises(_lib.NativeUnavailable, match="not built from the current"):
        _lib.load.__wrapped__("io_native")


def test_loader_accepts_matching_library():
    lib = _lib.load.__wrapped__("io_native")
    f = lib.mifx_src_hash
    f.restype = __import__("ctypes").c_char_p
    assert f().decode() == build.source_hash(build.CSRC / "io_native.cpp")
