#!/bin/bash
# gconv weight gradient over any C % 8 (tap-straddling column tiles): tests, deeper + standard PATE benches
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gconv.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wg8_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/wg8_tests.log | tail -6; grep -c PASSED gpurun_out/wg8_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_pate.py --steps 20 --teachers 250 --deeper --no-sequential > gpurun_out/pate_deep2.jsonl 2> gpurun_out/pate_deep2.err || { tail -20 gpurun_out/pate_deep2.err; exit 1; }
cat gpurun_out/pate_deep2.jsonl
timeout -k 10 400 python -u tools/bench_pate.py --steps 30 --teachers 250 --no-sequential > gpurun_out/pate_std2.jsonl 2> gpurun_out/pate_std2.err || { tail -20 gpurun_out/pate_std2.err; exit 1; }
cat gpurun_out/pate_std2.jsonl
