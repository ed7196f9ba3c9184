#!/bin/bash
# Round 6, batch 22: PMC pass over the 3x3 weight-gradient shapes (nine-tap kernel vs MIOpen): MFMA busy, LDS
# instructions / bank conflicts per kernel.
set -o pipefail
mkdir -p gpurun_out/r6
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/r6/pmc_c3 -o pmc -- python3 tools/bench_conv3_wgrad.py --iters 3 > gpurun_out/r6/pmc_c3.log 2>&1 || { tail -5 gpurun_out/r6/pmc_c3.log; exit 1; }
python3 tools/pmc_mfma_table.py gpurun_out/r6/pmc_c3/pmc_results.db --title "PMC: 3x3 weight gradients at B=256 (nine-tap kernel vs MIOpen igemm_wrw)" > gpurun_out/r6/conv3_wgrad_pmc.md
rm -rf gpurun_out/r6/pmc_c3
head -14 gpurun_out/r6/conv3_wgrad_pmc.md
echo done
