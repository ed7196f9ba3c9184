#!/bin/bash
# gconv 32-channel tiles + deeper PATE ensemble: tests, deeper bench (ensemble vs sequential, and MIOpen-only A/B)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gconv.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/deep_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/deep_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_pate.py --steps 20 --teachers 50,250 --deeper > gpurun_out/pate_deep.jsonl 2> gpurun_out/pate_deep.err || { tail -20 gpurun_out/pate_deep.err; exit 1; }
cat gpurun_out/pate_deep.jsonl
