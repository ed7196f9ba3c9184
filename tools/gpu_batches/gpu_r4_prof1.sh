set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_wide_deep.py tests/test_shuffle.py tests/test_dist_gpu.py tests/test_bench_launch.py > gpurun_out/r4_t4.log 2>&1 || { tail -40 gpurun_out/r4_t4.log; exit 1; }
tail -2 gpurun_out/r4_t4.log
for r in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b4.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b4.json')); print('bench', round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2))"
done
bash tools/prof_run.sh bench_r4a 300 -- python3 bench.py --steps 200 --warmup 20
cat gpurun_out/bench_r4a_kernels.md | head -14
