#!/bin/bash
# gconv strided forward + weight gradient (deeper ensemble stride-2 layers): tests, deeper + standard PATE benches
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gconv.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/st2_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/st2_tests.log | tail -6; grep -c PASSED gpurun_out/st2_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_pate.py --steps 20 --teachers 250 --deeper --no-sequential > gpurun_out/pate_deep3.jsonl 2> gpurun_out/pate_deep3.err || { tail -20 gpurun_out/pate_deep3.err; exit 1; }
cat gpurun_out/pate_deep3.jsonl
timeout -k 10 400 python -u tools/bench_pate.py --steps 30 --teachers 250 --no-sequential > gpurun_out/pate_std3.jsonl 2> gpurun_out/pate_std3.err || { tail -20 gpurun_out/pate_std3.err; exit 1; }
cat gpurun_out/pate_std3.jsonl
