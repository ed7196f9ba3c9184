#!/bin/bash
# Round 6, batch 5: LDS bank-conflict share of the fused attention kernels with 160-byte LDS rows (default) vs 144-byte
# rows (tools/bin/libattention_ld72.so), one rocprofv3 --pmc pass each over eager BERT-base steps.
set -o pipefail
mkdir -p gpurun_out/r6
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 240 rocprofv3 --pmc $P -d gpurun_out/r6/pmc_bert80 -o pmc -- python3 -m mifx.trainer.bert_trainer --steps 3 --warmup 1 --no-graph > gpurun_out/r6/pmc_bert80.log 2>&1 || { tail -5 gpurun_out/r6/pmc_bert80.log; exit 1; }
python3 tools/pmc_mfma_table.py gpurun_out/r6/pmc_bert80/pmc_results.db --title "PMC: BERT-base B=32 S=128 eager step, attention LDS rows 160 B (ATTN_LD_SHORT=80)" > gpurun_out/r6/bert_pmc_ld80.md
export MIFX_LIB_ATTENTION=$R/tools/bin/libattention_ld72.so
timeout -s KILL 240 rocprofv3 --pmc $P -d gpurun_out/r6/pmc_bert72 -o pmc -- python3 -m mifx.trainer.bert_trainer --steps 3 --warmup 1 --no-graph > gpurun_out/r6/pmc_bert72.log 2>&1 || { tail -5 gpurun_out/r6/pmc_bert72.log; exit 1; }
python3 tools/pmc_mfma_table.py gpurun_out/r6/pmc_bert72/pmc_results.db --title "PMC: BERT-base B=32 S=128 eager step, attention LDS rows 144 B (round-5 layout)" > gpurun_out/r6/bert_pmc_ld72.md
grep -E "attn|kernel" gpurun_out/r6/bert_pmc_ld80.md | head -5
grep -E "attn" gpurun_out/r6/bert_pmc_ld72.md | head -5
rm -rf gpurun_out/r6/pmc_bert80 gpurun_out/r6/pmc_bert72
echo done
