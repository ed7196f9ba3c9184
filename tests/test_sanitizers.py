"""Host-side sanitizers over the native runtime code: ASan + UBSan on the TFRecord codec (csrc/io_native.cpp), the
direct-RCCL argument paths against a stub RCCL (csrc/rccl_direct.cpp), and the multithreaded GBDT learner
(csrc/gbdt.cpp) under ASan + UBSan AND ThreadSanitizer. GPU sanitizers / xnack-on runs are unavailable on the MI355X
pool, so device kernels are covered by numerics + determinism tests instead."""
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


def _run(exe, args=(), **extra):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1", **extra)
    env.pop("LD_PRELOAD", None)
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=600, env=env)


def _build(cmd):
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_gbdt_learner_sanitizers(tmp_path, san):
    """Thread-count determinism, leaf / predict agreement and every buffer access of the tree learner, under
    ASan + UBSan and under TSan (features split over std::threads when n * f > 200k, rows in predict)."""
    exe = str(tmp_path / "gbdt_fuzz")
    _build(["g++", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-std=c++17", "-pthread",
            os.path.join(ROOT, "tools", "sanitize", "gbdt_fuzz.cpp"), os.path.join(ROOT, "csrc", "gbdt.cpp"),
            "-o", exe])
    r = _run(exe)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "240 trees, 0 failures" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_rccl_direct_argument_paths_asan_ubsan(tmp_path):
    stub, nosym, exe = (str(tmp_path / n) for n in ("librccl_stub.so", "librccl_nosym.so", "rccl_fuzz"))
    src = os.path.join(ROOT, "tools", "sanitize")
    _build(["g++", "-shared", "-fPIC", os.path.join(src, "rccl_stub.cpp"), "-o", stub])
    _build(["g++", "-shared", "-fPIC", "-DNO_ALLREDUCE", os.path.join(src, "rccl_stub.cpp"), "-o", nosym])
    _build(["g++", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-std=c++17",
            os.path.join(src, "rccl_direct_fuzz.cpp"), os.path.join(ROOT, "csrc", "rccl_direct.cpp"), "-ldl",
            "-o", exe])
    r = _run(exe, (stub, nosym))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
