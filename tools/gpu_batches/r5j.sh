# round 5: ResNet A/B with the implicit-GEMM 3x3 convolutions; DP peer-memory exchange diagnostics
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in 1 0; do
  MIFX_CONV3X3=$v timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5j_resnet_$v.json 2> gpurun_out/r5j_resnet_$v.err || { tail -20 gpurun_out/r5j_resnet_$v.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5j_resnet_$v.json') if l.startswith('{')][-1]); print('conv3x3', '$v', round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5j.md 2> gpurun_out/resnet_steady_r5j.err || { tail -5 gpurun_out/resnet_steady_r5j.err; exit 1; }
head -45 gpurun_out/resnet_steady_r5j.md
timeout -k 10 600 python -u -m pytest tests/test_tp_ipc.py -m gpu -x -q -k "fp32 or ddp_ipc" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5j_dp_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r5j_dp_tests.log; exit $rc
