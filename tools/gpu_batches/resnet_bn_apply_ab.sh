# round 5: BatchNorm + ReLU folded into the consumer 1x1 GEMM operands (AX / BNX) + BN apply passes with 4 rows in
# flight; tests; ResNet A/B (fold on/off, apply rows 8/16); steady table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_bn_fold.py tests/test_bn_relu.py tests/test_conv1x1.py tests/test_gemm8.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5x_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5x_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5x_tests.log | head -30; tail -40 gpurun_out/r5x_tests.log; exit $rc; }
for v in "MIFX_BN_FOLD=1" "MIFX_BN_FOLD=0" "MIFX_BN_FOLD=1 MIFX_BN_APPLY_ROWS=16" "MIFX_BN_FOLD=1" "MIFX_BN_FOLD=0" "MIFX_BN_FOLD=1 MIFX_BN_APPLY_ROWS=16"; do
  tag=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5x_resnet_$tag.json 2> gpurun_out/r5x_resnet_$tag.err || { tail -20 gpurun_out/r5x_resnet_$tag.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5x_resnet_$tag.json') if l.startswith('{')][-1]); print('$v', round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5x.md 2> gpurun_out/resnet_steady_r5x.err || { tail -5 gpurun_out/resnet_steady_r5x.err; exit 1; }
head -30 gpurun_out/resnet_steady_r5x.md
