#!/bin/bash
# Round 2: A/B early first fetch (production build) vs tools/bin/libwdc_base.so; RU=16 reduce (tools/bin/libwd_ru16.so)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2s.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_r2s.log; exit 1; }
tail -1 gpurun_out/pytest_r2s.log
for v in base early ru16 base2 early2; do
  unset MIFX_LIB_WD_CHAIN MIFX_LIB_WIDE_DEEP
  case $v in base*) export MIFX_LIB_WD_CHAIN=$PWD/tools/bin/libwdc_base.so;; ru16) export MIFX_LIB_WIDE_DEEP=$PWD/tools/bin/libwd_ru16.so;; esac
  timeout -k 10 200 python -u tools/ab_wd.py --kernels chain8 --batches 65536,131072 --rounds 3 > gpurun_out/ab_r2s_$v.txt 2>&1 || { tail -20 gpurun_out/ab_r2s_$v.txt; exit 1; }
  echo "== $v"; grep -v loss gpurun_out/ab_r2s_$v.txt | grep config
done
