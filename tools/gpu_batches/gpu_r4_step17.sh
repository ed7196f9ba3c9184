# Round-4 GPU batch 17: PMC counters of BERT-base's GEMMs at their routed kernels (two passes, each its own run).
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d gpurun_out/pmcg_r4_$i -o pmc -- python3 tools/pmc_gemm_probe.py --reps 10 > gpurun_out/pmcg_r4_$i.log 2>&1 || { tail -5 gpurun_out/pmcg_r4_$i.log; exit 1; }
  db=$(find gpurun_out/pmcg_r4_$i -name "*.db" | head -1)
  python3 tools/pmc_summary.py "$db" --out gpurun_out/gemm_pmc_r4_$i.md > /dev/null && rm -rf gpurun_out/pmcg_r4_$i
  echo "pmc pass $i ok"
done
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcg_r4_t -o kt -- python3 tools/pmc_gemm_probe.py --reps 10 > gpurun_out/pmcg_r4_t.log 2>&1 || { tail -5 gpurun_out/pmcg_r4_t.log; exit 1; }
true
head -30 gpurun_out/gemm_pmc_r4_1.md
