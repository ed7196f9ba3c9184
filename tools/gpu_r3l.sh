#!/bin/bash
# gconv prefetch depth A/B (MIFX_GCONV_PD 1/2/3): numerics at the default, microbench each depth, PATE bench
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gconv.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pd_tests.log 2>&1 || { tail -20 gpurun_out/pd_tests.log; exit 1; }
tail -1 gpurun_out/pd_tests.log
for pd in 1 2 3; do
  MIFX_GCONV_PD=$pd timeout -k 10 200 python -u tools/bench_gconv.py > gpurun_out/gconv_pd$pd.jsonl 2> gpurun_out/gconv_pd$pd.err || { tail -5 gpurun_out/gconv_pd$pd.err; exit 1; }
  echo "pd=$pd"; cat gpurun_out/gconv_pd$pd.jsonl
done
