#!/bin/bash
# Round-6 start: headline bench at the driver's shape + a rocprofv3 kernel table of the W&D step
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/bench0.json 2> gpurun_out/r6/bench0.err || { tail -20 gpurun_out/r6/bench0.err; exit 1; }
cat gpurun_out/r6/bench0.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof0 -o run -- python -u bench.py --gpus 1 --steps 200 --warmup 20 --ref-batch 0 > gpurun_out/r6/prof0.log 2>&1 || { tail -20 gpurun_out/r6/prof0.log; exit 1; }
find gpurun_out/r6/prof0 -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'head -12 {}'
