#!/bin/bash
# Round 6, batch 12: ResNet-50 stem convolution on the hand-written MFMA kernel (csrc/stem_conv.hip): numerics tests,
# then same-box A/B of the captured B=256 step against the MIOpen stem (MIFX_STEM=0), and its kernel time.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stem_conv.py \
  > gpurun_out/r6/b12_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b12_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b12_tests.log
bash tools/ab.sh -n 2 -t 400 -o stem hip miopen=MIFX_STEM=0 -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_stem -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_stem.log 2>&1 || { tail -20 gpurun_out/r6/prof_stem.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_stem/run_results.db --top 100 > gpurun_out/r6/resnet_census_stem.md
rm -rf gpurun_out/r6/prof_stem
head -1 gpurun_out/r6/resnet_census_stem.md
grep -E "stem|igemm" gpurun_out/r6/resnet_census_stem.md
echo done
