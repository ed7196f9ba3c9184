set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_shuffle.py tests/test_dist_gpu.py tests/test_image_pipeline.py tests/test_parallel_gpu.py tests/test_analyzers_quantiles.py > gpurun_out/r4_t2.log 2>&1 || { tail -40 gpurun_out/r4_t2.log; exit 1; }
tail -3 gpurun_out/r4_t2.log
for r in 1 2; do
for s in 24301 0; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --shuffle-seed $s > gpurun_out/r4_ab_$s.$r.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_ab_$s.$r.json')); print('seed $s run $r', round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2))"
done; done
