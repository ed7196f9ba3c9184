#!/bin/bash
# DP-SGD MNIST fused per-microbatch gradient kernel: numerics vs vmap, CNN bench (fused vs vmap), kernel trace;
# then the round-end rehearsal (full GPU suite, smoke, bench)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_privacy.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/dpm_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/dpm_tests.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_cnn.py --steps 30 --warmup 3 > gpurun_out/cnn_bench.jsonl 2> gpurun_out/cnn_bench.err || { tail -20 gpurun_out/cnn_bench.err; exit 1; }
cat gpurun_out/cnn_bench.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dpm_prof -o dpm -- python3 tools/bench_cnn.py --only dpsgd,dpsgd_vmap --steps 20 --warmup 2 > gpurun_out/dpm_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/dpm_prof.log; exit 1; }
bash tools/gpu_rehearsal.sh
