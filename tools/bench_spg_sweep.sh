#!/bin/bash
# bench.py at the driver's shape (20 timed steps) for several steps-per-graph values, alternating, 2 rounds
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for run in 1 2; do
  for spg in 5 10 20; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --steps-per-graph $spg --ref-batch 40 > gpurun_out/spg_$spg.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/spg_$spg.json'));print('spg',$spg,'run',$run,round(d['ms_per_step']*1e3,2),round(d['reference_batch']['ms_per_step']*1e3,2))"
  done
done
