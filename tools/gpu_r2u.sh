#!/bin/bash
# Round 2: xGMI exchange diagnostics (2 processes on one GPU)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u tools/xgmi_probe.py --world 2 --iters 50 --steps 8 > gpurun_out/xgmi_probe_r2u.log 2>&1 || { tail -30 gpurun_out/xgmi_probe_r2u.log; exit 1; }
timeout -k 10 180 python -u tools/xgmi_probe.py --world 4 --iters 50 --steps 8 > gpurun_out/xgmi_probe_r2u4.log 2>&1 || { tail -30 gpurun_out/xgmi_probe_r2u4.log; exit 1; }
grep -v "Gloo\|socket.cpp\|amdgpu.ids" gpurun_out/xgmi_probe_r2u4.log | grep "\[e\|\[g\|\[c\|stress"
grep -v "Gloo\|socket.cpp\|amdgpu.ids" gpurun_out/xgmi_probe_r2u.log
