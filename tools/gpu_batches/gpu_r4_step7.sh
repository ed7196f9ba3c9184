# Round-4 GPU batch 7: W&D per-phase stamps (T=256 included), NT kernel on the dX shapes vs hipBLASLt.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gemm.py -k "nn or dx" > gpurun_out/r4_t7n.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t7n.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/stamps_wdc.py --quick > gpurun_out/wdc_stamps_r4.txt 2>&1 || { tail -20 gpurun_out/wdc_stamps_r4.txt; exit 1; }
cat gpurun_out/wdc_stamps_r4.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u tools/bench_gemm_hip.py --dx > gpurun_out/gemm_dx_r4.jsonl 2> gpurun_out/gemm_dx_r4.err || { tail -5 gpurun_out/gemm_dx_r4.err; exit 1; }
cut -c1-160 gpurun_out/gemm_dx_r4.jsonl
timeout -k 10 400 python -u tools/torch_kernel_table.py --model bert --batch 32 --seq 128 --warmup 6 --active 3 > gpurun_out/bert_steady_r4.md 2> gpurun_out/bert_steady_r4.err || { tail -5 gpurun_out/bert_steady_r4.err; exit 1; }
head -n 30 gpurun_out/bert_steady_r4.md
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_parallel_gpu.py -k "resnet" > gpurun_out/r4_t7a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t7a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 5 > gpurun_out/resnet_steady_r4.md 2> gpurun_out/resnet_steady_r4.err || { tail -5 gpurun_out/resnet_steady_r4.err; exit 1; }
head -n 8 gpurun_out/resnet_steady_r4.md
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_r4.json 2> gpurun_out/resnet_r4.err || { tail -5 gpurun_out/resnet_r4.err; exit 1; }
cut -c1-300 gpurun_out/resnet_r4.json
timeout -k 10 600 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 --no-graph > gpurun_out/resnet_r4_eager.json 2> gpurun_out/resnet_r4_eager.err || { tail -5 gpurun_out/resnet_r4_eager.err; exit 1; }
cut -c1-300 gpurun_out/resnet_r4_eager.json
timeout -k 10 600 python -u tools/bench_resnet_convs.py > gpurun_out/resnet_conv_routes_r4.jsonl 2> gpurun_out/resnet_conv_routes_r4.err || { tail -5 gpurun_out/resnet_conv_routes_r4.err; exit 1; }
cut -c1-400 gpurun_out/resnet_conv_routes_r4.jsonl
