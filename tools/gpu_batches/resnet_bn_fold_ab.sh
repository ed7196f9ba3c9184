# round 5: BN fold (forward: in-place LDS operand transform; backward: activation re-derived by the BN backward apply for dW); tests; ResNet A/B

set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bn_fold.py tests/test_bn_relu.py tests/test_conv1x1.py tests/test_gemm8.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5za_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5za_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5za_tests.log | head -30; tail -40 gpurun_out/r5za_tests.log; exit $rc; }
for v in "MIFX_BN_FOLD=1" "MIFX_BN_FOLD=0" "MIFX_BN_FOLD=1" "MIFX_BN_FOLD=0" "MIFX_BN_FOLD=1 MIFX_BNX_DW=1"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5za_resnet_$tag.json 2> gpurun_out/r5za_resnet_$tag.err || { tail -20 gpurun_out/r5za_resnet_$tag.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5za_resnet_$tag.json') if l.startswith('{')][-1]); print('$v', round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
MIFX_BN_FOLD=1 timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5za.md 2> gpurun_out/resnet_steady_r5za.err || { tail -5 gpurun_out/resnet_steady_r5za.err; exit 1; }
head -30 gpurun_out/resnet_steady_r5za.md
