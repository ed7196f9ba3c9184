#!/bin/bash
# Round 6, batch 6: coalesced deferred flushes in the ResNet DP step (MIFX_DP_FLUSH_MIN_WG): DP rehearsal test,
# forced one-rank DP throughput at three thresholds vs single GPU, per-step census of the default.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  > gpurun_out/r6/b6_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r6/b6_tests.log | tail -30; tail -5 gpurun_out/r6/b6_tests.log; exit 1; }
tail -2 gpurun_out/r6/b6_tests.log
for t in 1024 2048 100000; do
  MIFX_DP_FORCE=1 MIFX_DP_FLUSH_MIN_WG=$t timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_dpf_$t.json 2> gpurun_out/r6/resnet_dpf_$t.err || { tail -20 gpurun_out/r6/resnet_dpf_$t.err; exit 1; }
  echo "min_wg $t: $(grep '^{' gpurun_out/r6/resnet_dpf_$t.json | tail -1 | cut -c1-160)"
done
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_1c.json 2> gpurun_out/r6/resnet_1c.err || { tail -20 gpurun_out/r6/resnet_1c.err; exit 1; }
echo "single: $(grep '^{' gpurun_out/r6/resnet_1c.json | tail -1 | cut -c1-160)"
MIFX_DP_FORCE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_dpfc -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_dpfc.log 2>&1 || { tail -20 gpurun_out/r6/prof_dpfc.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_dpfc/run_results.db --top 90 > gpurun_out/r6/census_dp_coalesced.md
rm -rf gpurun_out/r6/prof_dpfc
head -1 gpurun_out/r6/census_dp_coalesced.md
grep -E "tn_grouped|copyBuffer" gpurun_out/r6/census_dp_coalesced.md
echo done
