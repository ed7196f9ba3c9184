# Round-4 GPU batch 12: in-kernel record prefetch (tests + bench A/B at both batches).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 800 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_deep.py tests/test_shuffle.py tests/test_dist_gpu.py tests/test_bert_tp.py tests/test_tp_ipc.py -k "prefetch or large_tile or shuffle or xgmi or dist or embedding or bert or ipc" > gpurun_out/r4_t12a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t12a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
for pf in 1 0; do
MIFX_WD_PREFETCH=$pf timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b12.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b12.json')); print('selfprefetch', $pf, round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2), d['config']['grad_check_max_rel_err_vs_fp32'])" | tee -a gpurun_out/wd_selfprefetch_ab_r4.txt
done
done
