#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python -u tools/dp_step_overhead.py > gpurun_out/dp_overhead.log 2>&1; rc=$?
grep -E "batch|Error|error" gpurun_out/dp_overhead.log | head -12; exit $rc
