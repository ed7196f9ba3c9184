#!/bin/bash
# Round 2: conflict-free LDS row permutations in the chained kernel: tests, A/B, stamps, bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2o.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2o.log | tail -30; tail -5 gpurun_out/pytest_r2o.log; exit 1; }
tail -1 gpurun_out/pytest_r2o.log
timeout -k 10 300 python -u tools/ab_wd.py --kernels chain8,chain4 --batches 65536,131072 --rounds 3 > gpurun_out/ab_r2o.txt 2>&1 || { tail -20 gpurun_out/ab_r2o.txt; exit 1; }
cat gpurun_out/ab_r2o.txt
timeout -k 10 120 python -u tools/stamps_wdc.py > gpurun_out/stamps_r2o.txt 2>&1 || { tail -20 gpurun_out/stamps_r2o.txt; exit 1; }
tail -15 gpurun_out/stamps_r2o.txt
timeout -k 10 300 python -u bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_r2o_long.json 2> gpurun_out/bench_r2o_long.err || { tail -20 gpurun_out/bench_r2o_long.err; exit 1; }
cut -c1-200 gpurun_out/bench_r2o_long.json
