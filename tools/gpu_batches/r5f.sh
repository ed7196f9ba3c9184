# round 5: steady-state ResNet table on the fused path; headline bench sanity
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5b.md 2> gpurun_out/resnet_steady_r5b.err || { tail -5 gpurun_out/resnet_steady_r5b.err; exit 1; }
head -60 gpurun_out/resnet_steady_r5b.md
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r5f_bench.json 2> gpurun_out/r5f_bench.err || { tail -5 gpurun_out/r5f_bench.err; exit 1; }
tail -1 gpurun_out/r5f_bench.json | cut -c1-400
