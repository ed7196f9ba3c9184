set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_shuffle.py tests/test_wide_deep.py tests/test_taxi_dnn.py tests/test_bench_launch.py tests/test_trainer_dp.py > gpurun_out/r4_t1.log 2>&1 || { tail -40 gpurun_out/r4_t1.log; exit 1; }
tail -3 gpurun_out/r4_t1.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_shuf.json 2> gpurun_out/r4_bench_shuf.err || { tail -20 gpurun_out/r4_bench_shuf.err; exit 1; }
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --shuffle-seed 0 > gpurun_out/r4_bench_noshuf.json 2> gpurun_out/r4_bench_noshuf.err || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_bench_shuf2.json 2>> gpurun_out/r4_bench_shuf.err || exit 1
for f in r4_bench_shuf r4_bench_noshuf r4_bench_shuf2; do python -c "import json,sys; d=json.load(open('gpurun_out/$f.json')); print('$f', d['ms_per_step']*1e3, d['reference_batch']['ms_per_step']*1e3)"; done
