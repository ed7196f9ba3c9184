# ResNet-50 stem max-pool with one window per thread vs window pairs in the forward (MIFX_POOL_PAIR=0 / 1): pool tests, kernel bench, step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_bn_relu.py -m gpu -x -q -k "maxpool or pool" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/poolf_tests.log 2>&1 || { tail -30 gpurun_out/poolf_tests.log; exit 1; }
tail -1 gpurun_out/poolf_tests.log
for ev in 0 1 0 1; do
  MIFX_POOL_PAIR=$ev timeout -k 10 120 python -u tools/pool_bench.py || exit 1
done
for ev in 0 1 0 1; do
  MIFX_POOL_PAIR=$ev timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/poolf_resnet.json 2> gpurun_out/poolf_resnet.err || { tail -20 gpurun_out/poolf_resnet.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/poolf_resnet.json') if l.startswith('{')][-1]); print('pair', $ev, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
