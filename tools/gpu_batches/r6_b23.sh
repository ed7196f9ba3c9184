#!/bin/bash
# Round 6, batch 23: wave-specialised nine-tap 3x3 weight gradient (4 multiplying + 4 staging waves, double-buffered
# LDS, one workgroup per CU) vs the 4-wave build (tools/bin/libc3_nows.so) and 8 staging loads in flight
# (tools/bin/libc3_sb8.so): tests, per-shape times, ResNet step A/B.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_conv3_wgrad.py \
  > gpurun_out/r6/b23_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b23_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b23_tests.log
timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/c3ws_shapes.jsonl 2> gpurun_out/r6/c3ws_shapes.err || { tail -5 gpurun_out/r6/c3ws_shapes.err; exit 1; }
cat gpurun_out/r6/c3ws_shapes.jsonl | cut -c1-150
MIFX_LIB_CONV3_WGRAD=$R/tools/bin/libc3_nows.so timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/c3nows_shapes.jsonl 2>/dev/null || exit 1
grep nine gpurun_out/r6/c3nows_shapes.jsonl | cut -c1-150
MIFX_LIB_CONV3_WGRAD=$R/tools/bin/libc3_sb8.so timeout -k 10 200 python -u tools/bench_conv3_wgrad.py > gpurun_out/r6/c3sb8_shapes.jsonl 2>/dev/null || exit 1
grep nine gpurun_out/r6/c3sb8_shapes.jsonl | cut -c1-150
bash tools/ab.sh -n 2 -t 400 -o c3ws ws nows=MIFX_LIB_CONV3_WGRAD=tools/bin/libc3_nows.so -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
echo done
