# Round-4 GPU batch 19: ResNet-50 v2 folded inference (KN17): tests, n18 serving example, latency bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_resnet_infer.py tests/test_bn_relu.py > gpurun_out/r4_t19a.log 2>&1 || { tail -30 gpurun_out/r4_t19a.log; exit 1; }
tail -1 gpurun_out/r4_t19a.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_notebook_examples.py -k n18 > gpurun_out/r4_t19b.log 2>&1 || { tail -30 gpurun_out/r4_t19b.log; exit 1; }
tail -1 gpurun_out/r4_t19b.log
timeout -k 10 400 python -u tools/bench_resnet_infer.py --batches 1 8 32 > gpurun_out/resnet_infer_r4.jsonl 2> gpurun_out/resnet_infer.err || { tail -10 gpurun_out/resnet_infer.err; exit 1; }
cat gpurun_out/resnet_infer_r4.jsonl
# BatchNorm counters advanced by one kernel per forward (defer_batch_counts): ResNet GPU tests and the B=256 step
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k resnet > gpurun_out/r4_t19c.log 2>&1 || { tail -30 gpurun_out/r4_t19c.log; exit 1; }
tail -1 gpurun_out/r4_t19c.log
for r in 1 2; do
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_nbt.json 2> gpurun_out/resnet_nbt.err || { tail -5 gpurun_out/resnet_nbt.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/resnet_nbt.json') if l.startswith('{')][-1]; print('resnet nbt', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/resnet_nbt_r4.txt
done
