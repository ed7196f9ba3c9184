#!/bin/bash
# Round 6, batch 20: global average pool with a channels_last gradient: ResNet tests, step time, census.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv1x1.py tests/test_conv3x3.py tests/test_bn_relu.py tests/test_conv3_wgrad.py tests/test_stem_conv.py tests/test_resnet_infer.py tests/test_parallel_gpu.py \
  > gpurun_out/r6/b20_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b20_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b20_tests.log
for i in 1 2; do timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 2>/dev/null | tail -1; done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_c3 -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_c3.log 2>&1 || { tail -20 gpurun_out/r6/prof_c3.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_c3/run_results.db --top 100 > gpurun_out/r6/resnet_census_gap.md
rm -rf gpurun_out/r6/prof_c3
head -1 gpurun_out/r6/resnet_census_gap.md
grep -E "Fill|igemm" gpurun_out/r6/resnet_census_gap.md
echo done
