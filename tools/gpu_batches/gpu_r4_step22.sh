# Round-4 GPU batch 22: kernel table of the folded ResNet-50 inference at B=1 (where the 1.8 ms go).
set -o pipefail
mkdir -p gpurun_out
bash tools/prof_run.sh resnet_infer_b1 300 -- python3 tools/bench_resnet_infer.py --batches 1
head -30 gpurun_out/resnet_infer_b1_kernels.md
