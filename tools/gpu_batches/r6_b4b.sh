#!/bin/bash
# Round 6, batch 4b: per-step kernel census (tools/step_window.py) of the single-GPU and the forced one-rank DP ResNet
# step (summaries kept, trace databases deleted on the box), then batch 5 (attention PMC).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_1b -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_1b.log 2>&1 || { tail -20 gpurun_out/r6/prof_1b.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_1b/run_results.db --top 90 > gpurun_out/r6/census_single.md
rm -rf gpurun_out/r6/prof_1b
MIFX_DP_FORCE=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r6/prof_dpfb -o run -- python -u -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > gpurun_out/r6/prof_dpfb.log 2>&1 || { tail -20 gpurun_out/r6/prof_dpfb.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_dpfb/run_results.db --top 90 > gpurun_out/r6/census_dp.md
python tools/timeline.py gpurun_out/r6/prof_dpfb/run_results.db --last 700 > gpurun_out/r6/timeline_dp.txt 2>&1 || true
rm -rf gpurun_out/r6/prof_dpfb
head -1 gpurun_out/r6/census_single.md gpurun_out/r6/census_dp.md
bash tools/gpu_batches/r6_b5.sh
