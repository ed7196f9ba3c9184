#!/bin/bash
# Round 6: split-wait IPC exchange + deferred weight gradients under data parallelism.
#  1. GPU tests of the exchange (both wait placements, the co-residence hazard), the fused SGD fixes, the ResNet DP
#     rehearsal (2 ranks sharing the GPU, deferred dW on/off) and the BERT TP rehearsals (deferred dW now on)
#  2. ResNet-50 B=256: single GPU vs the forced one-rank DP step (hooks, per-bucket flushes, IPC exchange)
#  3. rocprofv3 kernel table of the forced DP step (expect no MIOpen igemm_wrw)
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_sgd_fused.py "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  > gpurun_out/r6/dp_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r6/dp_tests.log | tail -30; tail -5 gpurun_out/r6/dp_tests.log; exit 1; }
tail -3 gpurun_out/r6/dp_tests.log
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_1.json 2> gpurun_out/r6/resnet_1.err || { tail -20 gpurun_out/r6/resnet_1.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_1.json | tail -1
export MIFX_DP_FORCE=1
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_dpf.json 2> gpurun_out/r6/resnet_dpf.err || { tail -20 gpurun_out/r6/resnet_dpf.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_dpf.json | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_dpf -o run -- python -u -m mifx.trainer.resnet_trainer --steps 10 --warmup 4 > gpurun_out/r6/prof_dpf.log 2>&1 || { tail -20 gpurun_out/r6/prof_dpf.log; exit 1; }
echo done
