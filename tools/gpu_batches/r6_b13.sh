#!/bin/bash
# Round 6, batch 13: stem kernels v3 (forward: 8 output rows per workgroup, weight fragments straight into registers;
# new weight-gradient kernel) vs the same with MIOpen's weight gradient vs MIOpen for both; tests; kernel time.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stem_conv.py \
  > gpurun_out/r6/b13_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b13_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b13_tests.log
bash tools/ab.sh -n 2 -t 400 -o stem3 v3 v3_wg_miopen=MIFX_STEM_WGRAD=0 miopen=MIFX_STEM=0 -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_stem3 -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_stem3.log 2>&1 || { tail -20 gpurun_out/r6/prof_stem3.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_stem3/run_results.db --top 100 > gpurun_out/r6/resnet_census_stem3.md
rm -rf gpurun_out/r6/prof_stem3
head -1 gpurun_out/r6/resnet_census_stem3.md
grep -E "stem" gpurun_out/r6/resnet_census_stem3.md
echo done
