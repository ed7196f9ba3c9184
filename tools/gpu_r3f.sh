#!/bin/bash
# Grouped MFMA conv (csrc/gconv.hip): numerics, microbench vs MIOpen, PATE ensemble tests + bench + trace
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gconv.py tests/test_pate_training.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gconv_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/gconv_tests.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gconv.py > gpurun_out/gconv_bench.jsonl 2> gpurun_out/gconv_bench.err || { tail -20 gpurun_out/gconv_bench.err; exit 1; }
cat gpurun_out/gconv_bench.jsonl
timeout -k 10 600 python -u tools/bench_pate.py --steps 30 > gpurun_out/pate_bench2.jsonl 2> gpurun_out/pate_bench2.err || { tail -20 gpurun_out/pate_bench2.err; exit 1; }
cat gpurun_out/pate_bench2.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pate_prof2 -o pate -- python3 tools/bench_pate.py --steps 12 --teachers 250 > gpurun_out/pate_prof2.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/pate_prof2.log; exit 1; }
echo done
