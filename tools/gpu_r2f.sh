#!/bin/bash
# Round 2: chained W&D kernel with weight-image pad 16: numerics, A/B (4 vs 8 waves vs tile), SQ counters
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_wide_deep.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r2f.log 2>&1 || { echo "pytest failed"; grep -E "Error|assert|FAILED|error" gpurun_out/pytest_r2f.log | tail -30; tail -5 gpurun_out/pytest_r2f.log; exit 1; }
tail -2 gpurun_out/pytest_r2f.log
timeout -k 10 300 python -u tools/ab_wd.py --batches 65536,131072,40 > gpurun_out/ab_r2f.jsonl 2> gpurun_out/ab_r2f.err || { tail -20 gpurun_out/ab_r2f.err; exit 1; }
cat gpurun_out/ab_r2f.jsonl
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for k in chain8 chain4; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_r2f_$k -o pmc -- python3 tools/ab_wd.py --kernels $k --batches 65536 --rounds 1 > gpurun_out/pmc_r2f_$k.log 2>&1 || { tail -20 gpurun_out/pmc_r2f_$k.log; exit 1; }
python3 tools/pmc_summary.py $(find gpurun_out/pmc_r2f_$k -name "*.db" | head -1) --match wdc_fused --out gpurun_out/pmc_r2f_$k.md
done
