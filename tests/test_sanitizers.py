"""Host-side sanitizers (ASan + UBSan) over the native runtime code (csrc/io_native.cpp).
GPU sanitizers / xnack-on runs are unavailable on the MI355X pool, so device kernels are covered by
numerics + determinism tests instead."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.join(os.path.dirname(__file__), "..")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_io_native_asan_ubsan_fuzz(tmp_path):
    exe = str(tmp_path / "io_fuzz")
    cmd = ["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-std=c++17",
           os.path.join(ROOT, "tools", "sanitize", "io_native_fuzz.cpp"), os.path.join(ROOT, "csrc", "io_native.cpp"),
           "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
