# ResNet-50 stem max-pool with general gather backward vs the 2x2-block backward (MIFX_POOL_EVEN=0 / 1): pool tests, kernel bench, step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_bn_relu.py -m gpu -x -q -k maxpool --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pool_tests.log 2>&1 || { tail -30 gpurun_out/pool_tests.log; exit 1; }
tail -1 gpurun_out/pool_tests.log
for ev in 0 1 0 1; do
  MIFX_POOL_EVEN=$ev timeout -k 10 120 python -u tools/pool_bench.py || exit 1
done
for ev in 0 1 0 1; do
  MIFX_POOL_EVEN=$ev timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/pool_resnet.json 2> gpurun_out/pool_resnet.err || { tail -20 gpurun_out/pool_resnet.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/pool_resnet.json') if l.startswith('{')][-1]); print('even', $ev, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
