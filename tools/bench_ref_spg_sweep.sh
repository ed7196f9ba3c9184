set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
for run in 1 2 3; do
  for v in 20 50 100; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --ref-steps-per-graph $v > gpurun_out/refspg_$v$run.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/refspg_$v$run.json'));print('refspg',$v,$run,round(d['ms_per_step']*1e3,2),round(d['reference_batch']['ms_per_step']*1e3,2))"
  done
done
