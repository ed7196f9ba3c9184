#!/bin/bash
# Round 6, batch 8: tests of this session's changes (gemm8 forward route, DP rehearsal at the new default, 8-rank SP
# rehearsal), forced-DP ResNet at the default, BERT forward-projection A/B (TunableOp table / heuristics / gemm8).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  "tests/test_gemm8.py::test_forward_route_to_gemm8_matches_fp32" \
  "tests/test_parallel_gpu.py::test_resnet50_dp2_on_gpu_replicas_identical_and_match_single" \
  "tests/test_tp_ipc.py::test_bert_sequence_parallel_captured_bit_identical_and_tracks_tp" \
  > gpurun_out/r6/b8_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|^E " gpurun_out/r6/b8_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r6/b8_tests.log
MIFX_DP_FORCE=1 timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 25 --warmup 5 > gpurun_out/r6/resnet_dpf_default.json 2> gpurun_out/r6/resnet_dpf_default.err || { tail -20 gpurun_out/r6/resnet_dpf_default.err; exit 1; }
echo "forced DP default: $(grep '^{' gpurun_out/r6/resnet_dpf_default.json | tail -1 | cut -c1-200)"
bash tools/ab.sh -n 2 -t 300 -o bert_fwd base notable=MIFX_BERT_GEMM_TABLE=0 g8=MIFX_G8_FWD=1 \
  g8b=MIFX_G8_FWD=4096:2304:768=0+4096:3072:768=0+4096:768:3072=5 \
  g8q=MIFX_G8_FWD=4096:2304:768=0 -- python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 || exit 1
echo done
