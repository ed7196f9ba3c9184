# gemm8 tile table for ResNet-50's 1x1 products (MIFX_G8_TUNED=1: measured winners, 0: throughput heuristic); tests; A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv1x1.py tests/test_resnet_infer.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g8t_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/g8t_tests.log | head -20; tail -20 gpurun_out/g8t_tests.log; exit 1; }
tail -1 gpurun_out/g8t_tests.log
bash tools/ab.sh -n 2 -t 400 -o g8tuned tuned heur=MIFX_G8_TUNED=0 -- python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5
