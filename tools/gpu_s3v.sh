#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s3v.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|PASSED" gpurun_out/pytest_s3v.log | tail -20; exit 1; }
tail -2 gpurun_out/pytest_s3v.log
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 1 --steps 100 --warmup 10 > gpurun_out/bench_s3v.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_s3v.log; exit 1; }
tail -1 gpurun_out/bench_s3v.log | cut -c1-200
