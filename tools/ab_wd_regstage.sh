set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for run in 1 2; do
  for v in dma reg; do
    if [ $v = reg ]; then export MIFX_LIB_WD_CHAIN=$PWD/tools/bin/libwd_chain_regstage.so MIFX_LIB_WD_CHAIN64=$PWD/tools/bin/libwd_chain64_regstage.so; else unset MIFX_LIB_WD_CHAIN MIFX_LIB_WD_CHAIN64; fi
    timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 > gpurun_out/abreg_$v$run.json 2>gpurun_out/abreg_err.log || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abreg_$v$run.json'));print('$v',$run,d['ms_per_step']*1e3,d['reference_batch']['ms_per_step']*1e3)"
  done
done
