#!/bin/bash
# native exp/log LRN, 1x1 wgrad as batched GEMM: tests, PATE bench, trace
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gconv.py tests/test_cnn_ops.py tests/test_pate_training.py tests/test_bn_relu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/k_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/k_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/bench_pate.py --steps 30 > gpurun_out/pate_bench10.jsonl 2> gpurun_out/pate_bench10.err || { tail -20 gpurun_out/pate_bench10.err; exit 1; }
cat gpurun_out/pate_bench10.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pate_prof9 -o pate -- python3 tools/bench_pate.py --steps 12 --teachers 250 --no-sequential > gpurun_out/pate_prof9.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/pate_prof9.log; exit 1; }
