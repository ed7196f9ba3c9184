#!/bin/bash
# Round 6, batch 21: W&D one-launch residue-class tail (MIFX_WD_RES_FUSED=1): bit-identity test vs the two-launch
# default, same-box bench A/B.
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_wide_deep.py -k "res_reduce_fused or run_to_run or xcd" \
  > gpurun_out/r6/b21_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|^E " gpurun_out/r6/b21_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/b21_tests.log
bash tools/ab.sh -n 3 -t 200 -o wdfused base fused=MIFX_WD_RES_FUSED=1 -- python -u bench.py --steps 200 --warmup 20 || exit 1
echo done
