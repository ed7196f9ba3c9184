#!/bin/bash
# Round 6, batch 15: nine-tap 3x3 weight-gradient kernel: tests vs fp32, per-shape time vs MIOpen, ResNet step A/B,
# kernel census.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3_wgrad.py \
  > gpurun_out/r6/b15_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b15_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b15_tests.log
timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/conv3_wgrad_shapes.jsonl 2> gpurun_out/r6/conv3_wgrad_shapes.err || { tail -5 gpurun_out/r6/conv3_wgrad_shapes.err; exit 1; }
cat gpurun_out/r6/conv3_wgrad_shapes.jsonl
bash tools/ab.sh -n 2 -t 400 -o c3wg c3 miopen=MIFX_CONV3_WGRAD=0 -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_c3 -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_c3.log 2>&1 || { tail -20 gpurun_out/r6/prof_c3.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_c3/run_results.db --top 100 > gpurun_out/r6/resnet_census_c3.md
rm -rf gpurun_out/r6/prof_c3
head -1 gpurun_out/r6/resnet_census_c3.md
grep -E "conv3_wgrad|igemm|stem" gpurun_out/r6/resnet_census_c3.md
echo done
