#!/bin/bash
# KFP taxi DNN: graph-capturable step (device batch selection, in-kernel row dedup): tests, bench, kernel trace
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_taxi_dnn.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/tdnn_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/tdnn_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_taxi_dnn.py > gpurun_out/tdnn_bench.jsonl 2>gpurun_out/tdnn_bench.err && cat gpurun_out/tdnn_bench.jsonl &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tdnn_prof -o tdnn -- python3 tools/bench_taxi_dnn.py --steps 600 > gpurun_out/tdnn_prof.log 2>&1; echo "prof rc=$?"
find gpurun_out/tdnn_prof -name "*kernel_stats.csv" | head -3
