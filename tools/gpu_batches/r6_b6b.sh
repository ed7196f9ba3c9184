#!/bin/bash
# Round 6, batch 6b: coalesced DP flushes diverged at B=256 (loss NaN at MIFX_DP_FLUSH_MIN_WG=1024): the 2-rank DP
# rehearsal with thresholds low enough that the tiny test model coalesces (and 0 = per bucket).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for t in 0 16 64; do
  MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
    > gpurun_out/r6/b6b_tests_$t.log 2>&1 && echo "threshold $t: pass" || { echo "threshold $t: FAIL"; grep -E "^E " gpurun_out/r6/b6b_tests_$t.log | head -8; }
done
echo done
