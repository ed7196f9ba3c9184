#!/bin/bash
# ResNet DP=2 exactness test + ResNet-50 throughput with default vs deterministic MIOpen solvers
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_parallel_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k resnet > gpurun_out/par_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|^E " gpurun_out/par_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_default.json 2> gpurun_out/resnet_default.err && tail -1 gpurun_out/resnet_default.json &&
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 --deterministic > gpurun_out/resnet_det.json 2> gpurun_out/resnet_det.err && tail -1 gpurun_out/resnet_det.json
