# Round-4 GPU batch 18: steady-state ResNet-50 kernel table on the routed default step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 4 > gpurun_out/resnet_steady_r4b.md 2> gpurun_out/resnet_table.err || { tail -5 gpurun_out/resnet_table.err; exit 1; }
head -40 gpurun_out/resnet_steady_r4b.md
