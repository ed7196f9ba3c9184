#!/bin/bash
# Round 6, batch 26: stem forward with 12 / 16 output rows per workgroup (tools/bin/libstem_r12.so, libstem_r16.so) vs
# 8 (default): numerics of the variants, ResNet step A/B.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
for v in r12 r16; do
  MIFX_LIB_STEM_CONV=$R/tools/bin/libstem_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_stem_conv.py > gpurun_out/r6/b26_$v.log 2>&1 || { echo "tests $v failed"; grep -E "FAILED|^E " gpurun_out/r6/b26_$v.log | tail -10; exit 1; }
  tail -1 gpurun_out/r6/b26_$v.log
done
bash tools/ab.sh -n 2 -t 400 -o stemrows r8 r12=MIFX_LIB_STEM_CONV=tools/bin/libstem_r12.so r16=MIFX_LIB_STEM_CONV=tools/bin/libstem_r16.so -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
echo done
