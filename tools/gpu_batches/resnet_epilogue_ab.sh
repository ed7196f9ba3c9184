# gemm8 staged epilogue: 8 rows' global operand loads in flight (new) vs one per row (old library); tests; ResNet A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm8.py tests/test_conv1x1.py tests/test_conv3x3.py tests/test_bn_fold.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/epi_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/epi_tests.log | head -20; tail -20 gpurun_out/epi_tests.log; exit 1; }
tail -1 gpurun_out/epi_tests.log
bash tools/ab.sh -n 2 -t 400 -o epi new old=MIFX_LIB_GEMM8=tools/bin/libmifx_gemm8_old.so -- python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5
