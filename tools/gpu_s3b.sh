#!/bin/bash
# Fused reduce+optimizer: W&D GPU tests, bench, rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3b.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_s3b.log; exit 1; }
tail -3 gpurun_out/pytest_s3b.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_s3b.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_s3b.log; exit 1; }
tail -1 gpurun_out/bench_s3b.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_wd3 -o wd -- python bench.py --steps 100 --warmup 10 --ref-steps 500 > gpurun_out/prof_wd3.log 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof_wd3.log; exit 1; }
find gpurun_out/prof_wd3 -name "*stats*"
