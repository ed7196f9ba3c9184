#!/bin/bash
# Round 6, batch 11: BatchNorm tile-statistics finalize in one launch (last-arriving group merges): numerics tests,
# ResNet-50 A/B vs the two-launch form; BERT TP=4 + sequence parallelism through the trainer (ranks sharing the GPU).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_bn_relu.py tests/test_conv1x1.py tests/test_bn_fold.py tests/test_conv3x3.py \
  "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  > gpurun_out/r6/b11_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b11_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b11_tests.log
bash tools/ab.sh -n 2 -t 400 -o bn_one one two=MIFX_BN_TILES_TWO_LAUNCH=1 -- python -u -m mifx.trainer.resnet_trainer --steps 30 --warmup 5 || exit 1
MIFX_SHARED_GPU=1 MIFX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29631 -m mifx.trainer.bert_trainer --layers 2 --steps 10 --warmup 3 \
  --sequence-parallel > gpurun_out/r6/bert_tp4_sp.json 2> gpurun_out/r6/bert_tp4_sp.err || { tail -20 gpurun_out/r6/bert_tp4_sp.err; exit 1; }
grep '^{' gpurun_out/r6/bert_tp4_sp.json | tail -1 | cut -c1-300
echo done
