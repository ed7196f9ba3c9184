#!/bin/bash
# fused-vs-unfused ResNet divergence diag; analyzer microbench + rocprof kernel stats.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/diag/bn_model_divergence.py > gpurun_out/diag_bn_div.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/diag_bn_div.log; exit 1; }
cat gpurun_out/diag_bn_div.log
timeout -k 10 300 python -u tools/bench_analyzers.py --rows 1048576 > gpurun_out/bench_analyzers.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_analyzers.log; exit 1; }
cat gpurun_out/bench_analyzers.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_an -o an -- python tools/bench_analyzers.py --rows 1048576 > gpurun_out/prof_an.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof_an.log; exit 1; }
find gpurun_out/prof_an -name "*kernel_stats*"
