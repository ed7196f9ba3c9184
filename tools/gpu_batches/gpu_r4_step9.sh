# Round-4 GPU batch 9: ResNet graph / routed-dgrad tests, ResNet routed A/B, W&D PMC passes.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k "resnet" > gpurun_out/r4_t9a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t9a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
for m in routed 0; do
MIFX_RESNET_HIP_CONV=$m timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_ab.json 2> gpurun_out/resnet_ab.err || { tail -5 gpurun_out/resnet_ab.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/resnet_ab.json') if l.startswith('{')][-1]; print('conv', '$m', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/resnet_routed_ab_r4.txt
done
done
bash tools/gpu_batches/gpu_r4_pmc.sh
