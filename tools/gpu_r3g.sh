#!/bin/bash
# vectorised LRN kernels: CNN op tests, PATE ensemble tests + bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_cnn_ops.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/lrn_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/lrn_tests.log | head -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_pate.py --steps 30 > gpurun_out/pate_bench3.jsonl 2> gpurun_out/pate_bench3.err || { tail -20 gpurun_out/pate_bench3.err; exit 1; }
cat gpurun_out/pate_bench3.jsonl
