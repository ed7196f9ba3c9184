#!/bin/bash
# Round 6, batch 9: BERT-base input-gradient GEMMs on the 8-wave kernel (MIFX_G8_DX) vs the tuned gemm_nt<128,96>:
# numerics test, then same-box A/B of the captured step.
set -o pipefail
mkdir -p gpurun_out/r6
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider "tests/test_gemm8.py::test_dx_route_to_gemm8_matches_fp32" > gpurun_out/r6/b9_tests.log 2>&1 || { tail -30 gpurun_out/r6/b9_tests.log; exit 1; }
tail -1 gpurun_out/r6/b9_tests.log
bash tools/ab.sh -n 2 -t 300 -o bert_dx base \
  dx5=MIFX_G8_DX=4096:768:2304=5+4096:768:3072=5 \
  dx3=MIFX_G8_DX=4096:768:2304=3+4096:768:3072=3 \
  dx4=MIFX_G8_DX=4096:768:2304=4+4096:768:3072=4 \
  dxa=MIFX_G8_DX=4096:768:768=5 -- python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 || exit 1
echo done
