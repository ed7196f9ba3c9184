#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=tests/test_bn_relu.py::test_resnet_fused_blocks_match_fp64_reference
timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bn_new1.log 2>&1; rc=$?; echo "rc=$rc"; grep -E "stem|passed|failed" gpurun_out/bn_new1.log | head -8
