#!/bin/bash
# Round 2: chained W&D kernel phase stamps + SQ counters (one pass, kernel-trace only)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u tools/stamps_wdc.py > gpurun_out/stamps_wdc_r2d.txt 2>&1 || { tail -20 gpurun_out/stamps_wdc_r2d.txt; exit 1; }
cat gpurun_out/stamps_wdc_r2d.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_r2d -o pmc -- python3 tools/ab_wd.py --kernels chain --batches 65536 --rounds 1 > gpurun_out/pmc_r2d.log 2>&1 || { tail -20 gpurun_out/pmc_r2d.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_r2d/**/*counter_collection.csv", recursive=True)
print(f)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for row in csv.DictReader(open(f[0])):
    k = row["Kernel_Name"][:40]
    agg[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()}, "n", len(next(iter(d.values()))))
PY
