#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_taxi_dnn.py -x -q -p no:cacheprovider > gpurun_out/pytest_tdnn.log 2>&1 || { tail -60 gpurun_out/pytest_tdnn.log; exit 1; }
tail -2 gpurun_out/pytest_tdnn.log
timeout -k 10 300 python tools/bench_taxi_dnn.py --steps 3000 > gpurun_out/taxi_dnn_bench.log 2>&1 || { cat gpurun_out/taxi_dnn_bench.log; exit 1; }
cat gpurun_out/taxi_dnn_bench.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tdnn -o tdnn -- python3 tools/bench_taxi_dnn.py --steps 300 > gpurun_out/prof_tdnn.log 2>&1 || { tail -20 gpurun_out/prof_tdnn.log; exit 1; }
echo prof ok
