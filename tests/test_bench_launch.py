"""bench.py owns its ranks: `python bench.py --gpus N` with no torchrun env starts N processes itself and
reports n_gpus N; under torchrun a WORLD_SIZE that differs from --gpus is refused (the driver's 8-GPU run must
never time one GPU and call it eight). Reference: the job-owned replicas of
`notebooks/training-jobs/distributed-tensorflow-training-job.yaml:8-18`."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env_extra=None, timeout=400):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def _json_line(stdout: str) -> dict:
    lines = [ln for ln in stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, f"expected exactly one stdout line, got {lines!r}"
    return json.loads(lines[0])


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="CPU (gloo) variant")
def test_bench_gpus2_spawns_two_gloo_ranks():
    p = _bench(["--gpus", "2", "--steps", "3", "--warmup", "1", "--ref-steps", "3", "--batch-per-gpu", "512",
                "--data-per-gpu", "4096"])
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_line(p.stdout)
    assert out["n_gpus"] == 2 and out["world_size_seen_by_backend"] == 2 and out["backend"] == "gloo"
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 1024
    assert out["config"]["replicas_bit_identical"] is True
    assert len(out["config"]["dp_exchange_per_rank"]) == 2
    assert out["reference_batch"]["replicas_bit_identical"] is True


def test_bench_refuses_world_size_mismatch():
    p = _bench(["--gpus", "4", "--steps", "1"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert p.returncode == 2 and p.stdout.strip() == ""
    assert "refusing" in p.stderr


def test_bench_rank_failure_takes_the_job_down():
    """Rank 1 dies right after the rendezvous (fault injection); rank 0 would wait for it forever in the first
    collective: the launcher must kill it and fail the job with rank 1's code and no result line."""
    p = _bench(["--gpus", "2", "--steps", "1", "--batch-per-gpu", "256", "--data-per-gpu", "4096"],
               {"MIFX_BENCH_FAIL_RANK": "1"}, timeout=120)
    assert p.returncode == 3 and p.stdout.strip() == "", p.stderr[-2000:]
    assert "rank 1 exited with 3" in p.stderr


@pytest.mark.gpu
def test_bench_gpus2_shared_gpu_rehearsal():
    """The self-spawn entry point on one GPU: 2 ranks share cuda:0 over gloo (functional only), the xGMI exchange
    is set up, self-tested and validated after the timed region, and rank 0's single JSON line says dp2."""
    p = _bench(["--gpus", "2", "--steps", "10", "--warmup", "2", "--ref-steps", "50", "--batch-per-gpu", "8192",
                "--data-per-gpu", str(1 << 18)],
               {"MIFX_SHARED_GPU": "1", "MIFX_DIST_BACKEND": "gloo", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = _json_line(p.stdout)
    assert out["n_gpus"] == 2 and out["world_size_seen_by_backend"] == 2
    assert out["config"]["replicas_bit_identical"] is True
    assert all(d for d in out["config"]["dp_exchange_per_rank"])
