# round 5: MFMA utilisation of the ResNet-50 step's hand-written kernels (one rocprofv3 --pmc pass; MIOpen's
# first-call solver search excluded by the kernel filter)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $P -d gpurun_out/pmc_resnet -o pmc -- python3 -m mifx.trainer.resnet_trainer --steps 4 --warmup 2 --no-graph > gpurun_out/pmc_resnet.log 2>&1 || { tail -5 gpurun_out/pmc_resnet.log; exit 1; }
db=$(find gpurun_out/pmc_resnet -name "*.db" | head -1)
python3 tools/pmc_mfma_table.py "$db" --top 30 --match "gemm8_(nt|conv|tn)|bn_(apply|bwd|tiles|stats|finalize)|gconv_|weight_prep|maxpool_" --title "PMC: ResNet-50 B=256 training step (eager, 4 steps), hand-written kernels, MFMA utilisation" > gpurun_out/resnet_pmc_r5.md && rm -rf gpurun_out/pmc_resnet
head -36 gpurun_out/resnet_pmc_r5.md
