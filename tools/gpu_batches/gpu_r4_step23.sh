# Round-4 GPU batch 23: split-reduction gconv forward (batch-1 inference): conv / ResNet / PATE tests and the
# inference latency bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gconv.py tests/test_resnet_infer.py tests/test_privacy.py tests/test_parallel_gpu.py -k "gconv or split or folded or pate or resnet or conv or residual" > gpurun_out/r4_t23a.log 2>&1 || { tail -30 gpurun_out/r4_t23a.log; exit 1; }
tail -1 gpurun_out/r4_t23a.log
timeout -k 10 400 python -u tools/bench_resnet_infer.py --batches 1 8 32 > gpurun_out/resnet_infer_r4c.jsonl 2> gpurun_out/resnet_infer.err || { tail -10 gpurun_out/resnet_infer.err; exit 1; }
cat gpurun_out/resnet_infer_r4c.jsonl
