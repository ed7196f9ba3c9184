# round 5: 1x1 input gradients on the pipelined GEMM with the BatchNorm backward sums in its epilogue (EPI_BNBWD)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv1x1.py tests/test_gemm8.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5g_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5g_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5g_tests.log; exit $rc; }
for v in gemm8 miopen gemm8 miopen; do
  MIFX_CONV1X1_DGRAD=$v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5g_resnet_$v.json 2> gpurun_out/r5g_resnet_$v.err || { tail -20 gpurun_out/r5g_resnet_$v.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5g_resnet_$v.json') if l.startswith('{')][-1]); print('dgrad', '$v', round(r['value'],1), r.get('unit'), round(r.get('ms_per_step',0),3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5g.md 2> gpurun_out/resnet_steady_r5g.err || { tail -5 gpurun_out/resnet_steady_r5g.err; exit 1; }
head -50 gpurun_out/resnet_steady_r5g.md
