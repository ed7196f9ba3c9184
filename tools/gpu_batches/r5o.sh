# round 5: split-K chunk of the 1x1 weight gradients in the grouped launch (A/B on the ResNet step)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in 4096 2048 8192 4096 2048; do
  MIFX_WGRAD_CHUNK=$c timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5o_resnet_$c.json 2> gpurun_out/r5o_resnet_$c.err || { tail -20 gpurun_out/r5o_resnet_$c.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5o_resnet_$c.json') if l.startswith('{')][-1]); print('chunk', $c, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
