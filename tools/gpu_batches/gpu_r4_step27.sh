# Round-4 GPU batch 27: end-of-round kernel tables (BERT step, W&D step) for the evidence index.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 3 > gpurun_out/bert_steady_r4e.md 2> gpurun_out/bert_table.err || { tail -5 gpurun_out/bert_table.err; exit 1; }
head -12 gpurun_out/bert_steady_r4e.md
bash tools/prof_run.sh bench_r4_end 300 -- python3 bench.py --gpus 1 --steps 200 --warmup 20
head -12 gpurun_out/bench_r4_end_kernels.md
