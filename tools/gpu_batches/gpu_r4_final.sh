# Round-4 final GPU batch: the driver's tiers (full pytest -m gpu, smoke, 1-GPU bench) and the config 4 / 5 and
# inference benches on the final tree.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash tools/gpu_batches/gpu_rehearsal.sh || exit 1
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_final.json 2> gpurun_out/bert_final.err || { tail -5 gpurun_out/bert_final.err; exit 1; }
grep "^{" gpurun_out/bert_final.json | tail -1
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_final.json 2> gpurun_out/resnet_final.err || { tail -5 gpurun_out/resnet_final.err; exit 1; }
grep "^{" gpurun_out/resnet_final.json | tail -1
timeout -k 10 400 python -u tools/bench_resnet_infer.py --batches 1 8 32 > gpurun_out/resnet_infer_final.jsonl 2> gpurun_out/resnet_infer.err || { tail -10 gpurun_out/resnet_infer.err; exit 1; }
cat gpurun_out/resnet_infer_final.jsonl
