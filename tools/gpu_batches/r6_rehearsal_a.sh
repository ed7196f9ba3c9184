#!/bin/bash
# Round-6 rehearsal part A: the driver's GPU test tier (full `pytest -m gpu`), alone in one call.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1120 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rehearsal.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|^E " gpurun_out/pytest_rehearsal.log | tail -30; tail -5 gpurun_out/pytest_rehearsal.log; exit 1; }
tail -1 gpurun_out/pytest_rehearsal.log
