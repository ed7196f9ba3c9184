# round 5: conv3x3 after the occupancy-aware tile picker + per-problem chunks; tests; ResNet A/B + steady table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_conv3x3.py tests/test_conv1x1.py tests/test_gemm8.py tests/test_parallel_gpu.py tests/test_tp_ipc.py -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r5l_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5l_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5l_tests.log | head -30; tail -30 gpurun_out/r5l_tests.log; exit $rc; }
for v in 1 0 1 0; do
  MIFX_CONV3X3=$v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5l_resnet_$v.json 2> gpurun_out/r5l_resnet_$v.err || { tail -20 gpurun_out/r5l_resnet_$v.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5l_resnet_$v.json') if l.startswith('{')][-1]); print('conv3x3', '$v', round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5l.md 2> gpurun_out/resnet_steady_r5l.err || { tail -5 gpurun_out/resnet_steady_r5l.err; exit 1; }
head -50 gpurun_out/resnet_steady_r5l.md
