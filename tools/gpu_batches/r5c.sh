# round 5: BERT steady-state kernel table with deferred grouped weight gradients; BERT GPU tests; ResNet table
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 3 > gpurun_out/bert_steady_r5.md 2> gpurun_out/bert_steady_r5.err || { tail -5 gpurun_out/bert_steady_r5.err; exit 1; }
head -45 gpurun_out/bert_steady_r5.md
timeout -k 10 600 python -u -m pytest tests/test_bert_tp.py tests/test_bert_component.py tests/test_flat_adamw.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5c_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/torch_kernel_table.py --model resnet --batch 256 --warmup 8 --active 3 > gpurun_out/resnet_steady_r5.md 2> gpurun_out/resnet_steady_r5.err || { tail -5 gpurun_out/resnet_steady_r5.err; exit 1; }
head -60 gpurun_out/resnet_steady_r5.md
