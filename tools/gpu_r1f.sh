#!/bin/bash
# round-1 GPU session F: all GPU tests (vectorised LN/GELU kernels), BERT + ResNet benches,
# steady-state kernel tables, eager GEMM timing, PATE teacher throughput
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -m mifx.trainer.bert_trainer --batch 32 --seq 128 --steps 30 --warmup 5 > gpurun_out/bert_bench.log 2>&1 || { tail -30 gpurun_out/bert_bench.log; exit 1; }
tail -1 gpurun_out/bert_bench.log
timeout -k 10 600 python -m mifx.trainer.resnet_trainer --batch 256 --steps 20 --warmup 8 > gpurun_out/resnet_bench.log 2>&1 || { tail -30 gpurun_out/resnet_bench.log; exit 1; }
tail -1 gpurun_out/resnet_bench.log
timeout -k 10 600 python tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady.md 2>gpurun_out/resnet_steady.err || { tail -30 gpurun_out/resnet_steady.err; exit 1; }
head -3 gpurun_out/resnet_steady.md
timeout -k 10 600 python tools/torch_kernel_table.py --model bert --batch 32 --warmup 5 --active 5 > gpurun_out/bert_steady.md 2>gpurun_out/bert_steady.err || { tail -30 gpurun_out/bert_steady.err; exit 1; }
head -3 gpurun_out/bert_steady.md
timeout -k 10 300 python examples/notebooks/n16_eager_execution.py > gpurun_out/n16.log 2>&1 || { tail -30 gpurun_out/n16.log; exit 1; }
tail -1 gpurun_out/n16.log
timeout -k 10 600 python -m mifx.privacy.pate.train_teachers --dataset mnist --nb_teachers 10 --teacher_id 0 --max_steps 600 --train_dir /tmp/pate > gpurun_out/pate_teacher.log 2>&1 || { tail -30 gpurun_out/pate_teacher.log; exit 1; }
grep -E "step 500|Precision" gpurun_out/pate_teacher.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
