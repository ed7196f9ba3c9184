#!/bin/bash
# Round 2: fused reduce + xGMI exchange + optimizer kernel: probe (2 and 4 ranks on one GPU), DP tests, 1-GPU overhead
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u tools/xgmi_probe.py --world 2 --iters 300 --steps 8 > gpurun_out/xgmi_probe_r2w.log 2>&1 || { tail -30 gpurun_out/xgmi_probe_r2w.log; exit 1; }
grep -v "Gloo\|socket.cpp\|amdgpu.ids" gpurun_out/xgmi_probe_r2w.log | grep "stress\|\[e\|\[g\|\[c"
timeout -k 10 180 python -u tools/xgmi_probe.py --world 4 --iters 300 --steps 8 > gpurun_out/xgmi_probe_r2w4.log 2>&1 || { tail -30 gpurun_out/xgmi_probe_r2w4.log; exit 1; }
grep -v "Gloo\|socket.cpp\|amdgpu.ids" gpurun_out/xgmi_probe_r2w4.log | grep "stress\|\[e\|\[g\|\[c"
timeout -k 10 400 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2w.log 2>&1 || { echo "pytest failed"; grep -E "Error|error|assert|FAILED|Timeout" gpurun_out/pytest_r2w.log | tail -30; tail -20 gpurun_out/pytest_r2w.log; exit 1; }
grep -E "PASSED|FAILED" gpurun_out/pytest_r2w.log; tail -1 gpurun_out/pytest_r2w.log
timeout -k 10 300 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead_r2w.jsonl 2> gpurun_out/dp_overhead_r2w.err || { tail -20 gpurun_out/dp_overhead_r2w.err; exit 1; }
cat gpurun_out/dp_overhead_r2w.jsonl
