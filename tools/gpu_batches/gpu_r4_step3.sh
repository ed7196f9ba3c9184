set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_wide_deep.py -k "large_tile or small_tile or gradients_match" > gpurun_out/r4_t3.log 2>&1 || { tail -40 gpurun_out/r4_t3.log; exit 1; }
tail -3 gpurun_out/r4_t3.log
for r in 1 2; do
for v in "MIFX_WD_T256=1 S=24301" "MIFX_WD_T256=0 S=24301" "MIFX_WD_T256=1 S=0"; do
eval "export $v"
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --shuffle-seed $S > gpurun_out/r4_ab3.json 2>gpurun_out/r4_ab3.err || { tail -5 gpurun_out/r4_ab3.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4_ab3.json')); print('$v run $r', round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2), d['config']['grad_check_max_rel_err_vs_fp32'])"
done; done
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_parallel_gpu.py tests/test_image_pipeline.py tests/test_analyzers_quantiles.py > gpurun_out/r4_t3b.log 2>&1 || { tail -40 gpurun_out/r4_t3b.log; exit 1; }
tail -3 gpurun_out/r4_t3b.log
