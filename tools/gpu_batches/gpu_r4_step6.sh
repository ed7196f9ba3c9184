# Round-4 GPU batch 6: 4-rank shared-GPU bench rehearsal, TP=2 kernel table, long-sequence attention timings,
# ResNet-50 / BERT steady-state kernel tables and step rates. Each GPU step has its own time limit; the batch stops
# at the first failure.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k "resnet" > gpurun_out/r4_t6a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t6a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/bench_shared_rehearsal.sh 4 || exit 1
timeout -k 10 400 python -u tools/bench_attention.py --seq 128 256 384 512 --drop 0.1 0 --sdpa > gpurun_out/attn_long_r4.jsonl 2> gpurun_out/attn_long_r4.err || { tail -5 gpurun_out/attn_long_r4.err; exit 1; }
cat gpurun_out/attn_long_r4.jsonl | cut -c1-220
timeout -k 10 600 python -u tools/tp_kernel_table.py --tp 2 > gpurun_out/bert_tp2_kernels_r4.md 2> gpurun_out/bert_tp2_r4.err || { tail -20 gpurun_out/bert_tp2_r4.err; exit 1; }
head -n 12 gpurun_out/bert_tp2_kernels_r4.md; tail -n 3 gpurun_out/bert_tp2_kernels_r4.md
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_r4.json 2> gpurun_out/bert_r4.err || { tail -5 gpurun_out/bert_r4.err; exit 1; }
cut -c1-300 gpurun_out/bert_r4.json
timeout -k 10 600 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady_r4.md 2> gpurun_out/resnet_steady_r4.err || { tail -5 gpurun_out/resnet_steady_r4.err; exit 1; }
head -n 8 gpurun_out/resnet_steady_r4.md
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_r4.json 2> gpurun_out/resnet_r4.err || { tail -5 gpurun_out/resnet_r4.err; exit 1; }
cut -c1-300 gpurun_out/resnet_r4.json
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 --no-graph > gpurun_out/resnet_r4_eager.json 2> gpurun_out/resnet_r4_eager.err || { tail -5 gpurun_out/resnet_r4_eager.err; exit 1; }
cut -c1-300 gpurun_out/resnet_r4_eager.json
