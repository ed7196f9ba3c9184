#!/bin/bash
# Round 6, batch 7: BERT-base forward projections -- bundled TunableOp table vs library heuristics vs the 8-wave gemm8
# kernel (MIFX_G8_FWD) for QKV / FFN-in / FFN-out, whole captured step; GPU tests of the gemm8 forward route.
set -o pipefail
mkdir -p gpurun_out/r6
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "tests/test_gemm8.py::test_forward_route_to_gemm8_matches_fp32" > gpurun_out/r6/b7_tests.log 2>&1 || { tail -30 gpurun_out/r6/b7_tests.log; exit 1; }
tail -1 gpurun_out/r6/b7_tests.log
bash tools/ab.sh -n 2 -t 300 -o bert_fwd base notable=MIFX_BERT_GEMM_TABLE=0 g8=MIFX_G8_FWD=1 \
  g8b=MIFX_G8_FWD=4096:2304:768=0+4096:3072:768=0+4096:768:3072=5 \
  g8q=MIFX_G8_FWD=4096:2304:768=0 -- python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 || exit 1
echo done
