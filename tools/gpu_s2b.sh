#!/bin/bash
# ResNet fused-BN gradient conditioning check vs fp64, remaining GPU suite, smoke, bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/diag/resnet_grad_fp64.py > gpurun_out/diag_resnet_fp64.log 2>&1 || { echo "diag failed"; tail -30 gpurun_out/diag_resnet_fp64.log; exit 1; }
cat gpurun_out/diag_resnet_fp64.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_bn_relu.py::test_resnet_fused_blocks_match_unfused_reference > gpurun_out/pytest_gpu_s2b.log 2>&1 || { echo "pytest failed rc=$?"; tail -60 gpurun_out/pytest_gpu_s2b.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_s2b.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_s2b.log 2>&1 || { echo smoke failed; cat gpurun_out/smoke_s2b.log; exit 1; }
cat gpurun_out/smoke_s2b.log
timeout -k 10 400 python bench.py > gpurun_out/bench_s2b.log 2>&1 || { echo bench failed; tail -30 gpurun_out/bench_s2b.log; exit 1; }
tail -1 gpurun_out/bench_s2b.log
