#!/bin/bash
# Round 2: PMC passes on the chained W&D kernel (B=65536), 8 SQ counters max per pass
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > /tmp/avail.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" /tmp/avail.txt | sort -u | grep -E "LDS|MFMA|WAIT|BUSY|INSTS_V|INSTS_L|ACTIVE|CYCLES" > gpurun_out/sq_counters_gfx950.txt || true
wc -l gpurun_out/sq_counters_gfx950.txt
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_MEM_VIOLATIONS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH"; do
  i=$((i+1))
  ok=""
  for c in $set; do grep -qx "$c" gpurun_out/sq_counters_gfx950.txt && ok="$ok $c"; done
  echo "pass $i:$ok"
  [ -z "$ok" ] && continue
  timeout -s KILL 90 rocprofv3 --pmc $ok -d /tmp/pmc_zd_$i -o pmc -- python3 tools/ab_wd.py --kernels chain8 --batches 65536 --rounds 1 --steps-per-graph 1 > gpurun_out/pmc_r2zd_$i.log 2>&1 || { tail -5 gpurun_out/pmc_r2zd_$i.log; continue; }
  python3 tools/pmc_summary.py $(find /tmp/pmc_zd_$i -name "*.db" | head -1) --match wdc_fused --out gpurun_out/pmc_r2zd_$i.md | head -14
done
