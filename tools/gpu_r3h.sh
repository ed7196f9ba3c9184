#!/bin/bash
# DP-SGD: per-example workgroups for M < B; tests + CNN bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_privacy.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dpm_tests4.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/dpm_tests4.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_cnn.py --steps 30 --warmup 3 --only dpsgd,dpsgd_m32,sgd,sgd_fused > gpurun_out/cnn_bench4.jsonl 2> gpurun_out/cnn_bench4.err || { tail -20 gpurun_out/cnn_bench4.err; exit 1; }
cat gpurun_out/cnn_bench4.jsonl
