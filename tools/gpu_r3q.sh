#!/bin/bash
# W&D one-row optimizer kernel (wd_opt1_sc): W&D + DP GPU tests, bench (reference batch 40 in the same line)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_wide_deep.py tests/test_dist_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/wd1_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/wd1_tests.log | tail -6; grep -c PASSED gpurun_out/wd1_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_wd1_$i.json 2> gpurun_out/bench_wd1_$i.err || { tail -5 gpurun_out/bench_wd1_$i.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_wd1_$i.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,3), 'e9', round(d['ms_per_step']*1e3,2), 'us; ref B=40:', round(d['reference_batch']['examples_per_sec']/1e6,3), 'e6', round(d['reference_batch']['ms_per_step']*1e3,2), 'us')"
done
