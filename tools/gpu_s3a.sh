#!/bin/bash
# Round-end rehearsal: full GPU test suite, smoke(), default bench.py.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3t.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s3a.log; exit 1; }
tail -3 gpurun_out/pytest_s3t.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s3t.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke_s3a.log; exit 1; }
tail -1 gpurun_out/smoke_s3t.log
timeout -k 10 600 python -u bench.py > gpurun_out/bench_s3t.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_s3a.log; exit 1; }
tail -1 gpurun_out/bench_s3t.log
