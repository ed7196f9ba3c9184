#!/bin/bash
# Same-box A/B of the W&D bench between the in-tree chained-kernel libraries and diagnostic builds
# tools/bin/libwd_chain_$1.so + tools/bin/libwd_chain64_$1.so (MIFX_LIB_WD_CHAIN / MIFX_LIB_WD_CHAIN64), alternating
# processes; prints us/step at B=65536 (200 steps) and at the reference batch.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
V=$1
for run in 1 2 3; do
  for v in base $V; do
    if [ $v = base ]; then unset MIFX_LIB_WD_CHAIN MIFX_LIB_WD_CHAIN64
    else export MIFX_LIB_WD_CHAIN=$PWD/tools/bin/libwd_chain_$V.so MIFX_LIB_WD_CHAIN64=$PWD/tools/bin/libwd_chain64_$V.so; fi
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > gpurun_out/ablib_$v$run.json 2>gpurun_out/ablib_$v$run.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ablib_$v$run.json'));print('$v',$run,round(d['ms_per_step']*1e3,2),round(d['reference_batch']['ms_per_step']*1e3,2),d['config'].get('grad_check_max_rel_err_vs_fp32'))"
  done
done
