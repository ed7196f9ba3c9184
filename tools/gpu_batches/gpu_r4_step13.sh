# Round-4 GPU batch 13: BN reduction grid cap A/B on the ResNet-50 step; BN numerics tests.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MIFX_BN_BLOCKS_CAP=2048 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bn_relu.py > gpurun_out/r4_t13a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t13a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
for cap in 512 2048 1024; do
MIFX_BN_BLOCKS_CAP=$cap timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_bn.json 2> gpurun_out/resnet_bn.err || { tail -5 gpurun_out/resnet_bn.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/resnet_bn.json') if l.startswith('{')][-1]; print('bn_cap', $cap, round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/resnet_bn_cap_ab_r4.txt
done
done
