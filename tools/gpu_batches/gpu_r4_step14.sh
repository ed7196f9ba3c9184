# Round-4 GPU batch 14: W&D prologue split -- per-phase stamps of the production kernels vs the no-image builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/stamps_wdc.py --quick > gpurun_out/wdc_stamps_full.txt 2>&1 || { tail -5 gpurun_out/wdc_stamps_full.txt; exit 1; }
timeout -k 10 300 python -u tools/stamps_wdc.py --quick --nostep > gpurun_out/wdc_stamps_nostep.txt 2>&1 || { tail -5 gpurun_out/wdc_stamps_nostep.txt; exit 1; }
grep -E "==|prologue|kernel \(" gpurun_out/wdc_stamps_full.txt gpurun_out/wdc_stamps_nostep.txt
