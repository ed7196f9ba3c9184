#!/bin/bash
# Round 6, batch 25: stride-1 projection shortcut (ResNet stage 1) in the conv1 pair node: tests, step A/B vs the
# separate node (MIFX_PAIR_S1=0), census.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv1x1.py tests/test_bn_relu.py tests/test_conv3x3.py tests/test_parallel_gpu.py \
  > gpurun_out/r6/b25_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b25_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b25_tests.log
bash tools/ab.sh -n 2 -t 400 -o pairs1 pair sep=MIFX_PAIR_S1=0 -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_c3 -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_c3.log 2>&1 || { tail -20 gpurun_out/r6/prof_c3.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_c3/run_results.db --top 100 > gpurun_out/r6/resnet_census_pair.md
rm -rf gpurun_out/r6/prof_c3
head -1 gpurun_out/r6/resnet_census_pair.md
grep -E "CUDAFunctor_add|bn_bwd_reduce|igemm" gpurun_out/r6/resnet_census_pair.md
echo done
