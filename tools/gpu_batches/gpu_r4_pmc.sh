# PMC counters of the headline W&D step (two passes, each its own short run: no pass exceeds the per-block limits)
set -o pipefail
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd "$R"
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P -d gpurun_out/pmc_r4_$i -o pmc -- python3 bench.py --steps 10 --warmup 2 > gpurun_out/pmc_r4_$i.log 2>&1 || { tail -5 gpurun_out/pmc_r4_$i.log; exit 1; }
  db=$(find gpurun_out/pmc_r4_$i -name "*.db" | head -1)
  python3 tools/pmc_summary.py "$db" --out gpurun_out/wd_pmc_r4_$i.md > /dev/null && rm -rf gpurun_out/pmc_r4_$i
  echo "pmc pass $i ok"
done
cat gpurun_out/wd_pmc_r4_1.md gpurun_out/wd_pmc_r4_2.md | head -80
