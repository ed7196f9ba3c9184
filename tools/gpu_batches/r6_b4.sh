#!/bin/bash
# Round 6, batch 4: ResNet data-parallel step with every gradient written into the bucket views (BatchNorm dgamma /
# dbeta included, no per-step bucket memset): DP rehearsal test, single vs forced one-rank DP throughput, and per-step
# kernel census of both (tools/step_window.py).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  > gpurun_out/r6/b4_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r6/b4_tests.log | tail -30; tail -5 gpurun_out/r6/b4_tests.log; exit 1; }
tail -2 gpurun_out/r6/b4_tests.log
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_1b.json 2> gpurun_out/r6/resnet_1b.err || { tail -20 gpurun_out/r6/resnet_1b.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_1b.json | tail -1 | cut -c1-200
MIFX_DP_FORCE=1 timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_dpfb.json 2> gpurun_out/r6/resnet_dpfb.err || { tail -20 gpurun_out/r6/resnet_dpfb.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_dpfb.json | tail -1 | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_1b -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_1b.log 2>&1 || { tail -20 gpurun_out/r6/prof_1b.log; exit 1; }
export MIFX_DP_FORCE=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_dpfb -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_dpfb.log 2>&1 || { tail -20 gpurun_out/r6/prof_dpfb.log; exit 1; }
unset MIFX_DP_FORCE
python tools/step_window.py gpurun_out/r6/prof_1b/run_results.db | head -3
python tools/step_window.py gpurun_out/r6/prof_dpfb/run_results.db | head -3
echo done
