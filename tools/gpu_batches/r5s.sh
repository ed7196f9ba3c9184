# round 5: narrow (BN = 64) gemm8 tiles -- numerics, 3x3 64-channel routing data, ResNet A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gemm8.py tests/test_conv1x1.py tests/test_conv3x3.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5s_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5s_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/r5s_tests.log | head -30; tail -30 gpurun_out/r5s_tests.log; exit $rc; }
MIFX_CONV3X3_64=1 timeout -k 10 400 python -u tools/bench_conv3x3.py > gpurun_out/r5s_conv3x3.jsonl 2> gpurun_out/r5s_conv3x3.err || { tail -20 gpurun_out/r5s_conv3x3.err; exit 1; }
grep '"H": 56, "C": 64' gpurun_out/r5s_conv3x3.jsonl
for v in "1 0" "0 0" "1 1" "1 0" "0 0" "1 1"; do
  set -- $v
  MIFX_G8_NARROW=$1 MIFX_CONV3X3_64=$2 timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5s_resnet_$1$2.json 2> gpurun_out/r5s_resnet_$1$2.err || { tail -20 gpurun_out/r5s_resnet_$1$2.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5s_resnet_$1$2.json') if l.startswith('{')][-1]); print('narrow', $1, 'conv3x3_64', $2, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
