#!/bin/bash
# Round 6, batch 17: nine-tap 3x3 weight gradient, stride 2 with phase-split staging; 6 staging loads in flight
# (tools/bin/libc3_batch6.so) vs 4; ResNet step A/B with the stride-2 convolution on the kernel.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3_wgrad.py \
  > gpurun_out/r6/b17_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b17_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b17_tests.log
timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/conv3_wgrad_shapes3.jsonl 2> gpurun_out/r6/conv3_wgrad_shapes3.err || { tail -5 gpurun_out/r6/conv3_wgrad_shapes3.err; exit 1; }
cat gpurun_out/r6/conv3_wgrad_shapes3.jsonl
MIFX_LIB_CONV3_WGRAD=$R/tools/bin/libc3_batch6.so timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/conv3_wgrad_shapes_b6.jsonl 2> gpurun_out/r6/conv3_wgrad_shapes_b6.err || { tail -5 gpurun_out/r6/conv3_wgrad_shapes_b6.err; exit 1; }
grep nine gpurun_out/r6/conv3_wgrad_shapes_b6.jsonl
bash tools/ab.sh -n 2 -t 400 -o c3s2 s2=MIFX_CONV3_WGRAD_S2=1 base -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
echo done
