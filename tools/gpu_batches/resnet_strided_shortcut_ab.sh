# round 5: strided 1x1 shortcuts on the center-tap implicit GEMM (forward + deferred dW); tests; ResNet A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv_geo.py tests/test_gemm8.py tests/test_conv1x1.py tests/test_conv3x3.py tests/test_resnet_infer.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5v_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5v_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5v_tests.log | head -30; tail -30 gpurun_out/r5v_tests.log; exit $rc; }
for v in 1 0 1 0; do
  MIFX_SC_G8=$v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5v_resnet_$v.json 2> gpurun_out/r5v_resnet_$v.err || { tail -20 gpurun_out/r5v_resnet_$v.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5v_resnet_$v.json') if l.startswith('{')][-1]); print('sc_g8', $v, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5v.md 2> gpurun_out/resnet_steady_r5v.err || { tail -5 gpurun_out/resnet_steady_r5v.err; exit 1; }
head -40 gpurun_out/resnet_steady_r5v.md
