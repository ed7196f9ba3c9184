#!/bin/bash
# gconv reduction chunk per barrier A/B (MIFX_GCONV_BK 32/64): numerics at both, microbench each
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for bk in 32; do
  MIFX_GCONV_BK=$bk timeout -k 10 300 python -u -m pytest tests/test_gconv.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/bk_tests_$bk.log 2>&1 || { tail -20 gpurun_out/bk_tests_$bk.log; exit 1; }
  tail -1 gpurun_out/bk_tests_$bk.log
  MIFX_GCONV_BK=$bk timeout -k 10 200 python -u tools/bench_gconv.py > gpurun_out/gconv_bk$bk.jsonl 2> gpurun_out/gconv_bk$bk.err || { tail -5 gpurun_out/gconv_bk$bk.err; exit 1; }
  echo "bk=$bk"; cat gpurun_out/gconv_bk$bk.jsonl
done
