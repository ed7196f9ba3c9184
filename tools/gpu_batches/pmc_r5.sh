# round 5: MFMA utilisation per kernel (one rocprofv3 --pmc pass each) of the ResNet-50 and BERT-base steps (eager)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --pmc $P -d gpurun_out/pmc_resnet -o pmc -- python3 -m mifx.trainer.resnet_trainer --steps 2 --warmup 1 --no-graph > gpurun_out/pmc_resnet.log 2>&1 || { tail -5 gpurun_out/pmc_resnet.log; exit 1; }
db=$(find gpurun_out/pmc_resnet -name "*.db" | head -1)
python3 tools/pmc_mfma_table.py "$db" --title "PMC: ResNet-50 B=256 training step (eager, 3 steps), MFMA utilisation per kernel" > gpurun_out/resnet_pmc_r5.md && rm -rf gpurun_out/pmc_resnet
head -30 gpurun_out/resnet_pmc_r5.md
timeout -s KILL 240 rocprofv3 --pmc $P -d gpurun_out/pmc_bert -o pmc -- python3 -m mifx.trainer.bert_trainer --steps 3 --warmup 1 --no-graph > gpurun_out/pmc_bert.log 2>&1 || { tail -5 gpurun_out/pmc_bert.log; exit 1; }
db=$(find gpurun_out/pmc_bert -name "*.db" | head -1)
python3 tools/pmc_mfma_table.py "$db" --title "PMC: BERT-base B=32 S=128 training step (eager, 4 steps), MFMA utilisation per kernel" > gpurun_out/bert_pmc_r5.md && rm -rf gpurun_out/pmc_bert
head -30 gpurun_out/bert_pmc_r5.md
