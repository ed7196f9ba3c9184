#!/bin/bash
# Round 6, batch 2:
#  1. ResNet DP rehearsal (2 ranks sharing the GPU) with deferred dW (ipc / rccl) and without; fused attention vs fp32
#  2. ResNet-50 B=256: single GPU vs the forced one-rank DP step; rocprofv3 kernel table of the forced DP step
#  3. W&D headline A/B: XCD-local reduction (xcd_of + XCD ordering) vs the residue-class reduction (MIFX_WD_RES=1)
#  4. BERT-base A/B: short attention kernels with 160-B LDS rows (new) vs 144-B rows (tools/bin/libattention_ld72.so)
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ "$SKIP_TESTS" = 1 ] || { timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  "tests/test_bert_tp.py::test_fused_attention_gpu" \
  > gpurun_out/r6/b2_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r6/b2_tests.log | tail -30; tail -5 gpurun_out/r6/b2_tests.log; exit 1; }
  tail -2 gpurun_out/r6/b2_tests.log; }
timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_1.json 2> gpurun_out/r6/resnet_1.err || { tail -20 gpurun_out/r6/resnet_1.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_1.json | tail -1
MIFX_DP_FORCE=1 timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r6/resnet_dpf.json 2> gpurun_out/r6/resnet_dpf.err || { tail -20 gpurun_out/r6/resnet_dpf.err; exit 1; }
grep '^{' gpurun_out/r6/resnet_dpf.json | tail -1
export MIFX_DP_FORCE=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_dpf -o run -- python -u -m mifx.trainer.resnet_trainer --steps 10 --warmup 4 > gpurun_out/r6/prof_dpf.log 2>&1 || { tail -20 gpurun_out/r6/prof_dpf.log; exit 1; }
unset MIFX_DP_FORCE
bash tools/ab.sh -n 3 -t 200 -o wd_res xcd res=MIFX_WD_RES=1 -- python -u bench.py --steps 20 --warmup 5 || exit 1
bash tools/ab.sh -n 2 -t 300 -o bert_ld ld80 ld72=MIFX_LIB_ATTENTION=tools/bin/libattention_ld72.so -- python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 || exit 1
echo done
