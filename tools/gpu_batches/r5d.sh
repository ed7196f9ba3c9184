# round 5: gemm8 staged epilogue / split-K grouped TN / fused 1x1 ResNet path: tests, then ResNet A/B and tables
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T() { timeout -k 10 "$1" python -u -m pytest "${@:2}" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider; }
T 600 tests/test_gemm8.py tests/test_conv1x1.py tests/test_bn_relu.py > gpurun_out/r5d_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r5d_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "1 1" "0 0" "1 0" "1 1"; do
  set -- $v
  MIFX_RESNET_FUSED_1X1=$1 MIFX_DEFER_DW=$2 timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5d_resnet_$1$2.json 2> gpurun_out/r5d_resnet_$1$2.err || { tail -20 gpurun_out/r5d_resnet_$1$2.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5d_resnet_$1$2.json') if l.startswith('{')][-1]); print('fused', $1, 'defer', $2, round(r['value'],1), r.get('unit'), round(r.get('ms_per_step',0),3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5.md 2> gpurun_out/resnet_steady_r5.err || { tail -5 gpurun_out/resnet_steady_r5.err; exit 1; }
head -50 gpurun_out/resnet_steady_r5.md
timeout -k 10 300 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 3 > gpurun_out/bert_steady_r5.md 2> gpurun_out/bert_steady_r5.err || { tail -5 gpurun_out/bert_steady_r5.err; exit 1; }
head -40 gpurun_out/bert_steady_r5.md
