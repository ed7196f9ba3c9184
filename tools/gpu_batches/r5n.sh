# round 5: BN tile-statistics kernels with more loads in flight; sources of the remaining small kernels
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv1x1.py tests/test_conv3x3.py tests/test_bn_relu.py tests/test_tp_ipc.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5n_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5n_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5n_tests.log | head -30; tail -30 gpurun_out/r5n_tests.log; exit $rc; }
timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5n_resnet.json 2> gpurun_out/r5n_resnet.err || { tail -20 gpurun_out/r5n_resnet.err; exit 1; }
python -c "import json; r=json.loads([l for l in open('gpurun_out/r5n_resnet.json') if l.startswith('{')][-1]); print('resnet', round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 6 --active 2 --sources FillFunctor,elementwise_kernel_manual_unroll,bfloat16_copy,SubTensorOp,bn_bwd_reduce,bn_stats > gpurun_out/r5n_sources.md 2> gpurun_out/r5n_sources.err || { tail -5 gpurun_out/r5n_sources.err; exit 1; }
cat gpurun_out/r5n_sources.md | cut -c1-400
