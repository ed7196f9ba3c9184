# Round-4 GPU batch: TP IPC, W&D / shuffle / dist / bench-launch / BERT-TP / GEMM / image tests, two bench runs and a
# rocprof kernel table. A test FAILURE (pytest rc 1) does not stop the batch; a fault, abort or time limit does.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run_tests() {  # log, timeout, files...
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests $log rc=$rc: stopping"; exit $rc; fi
  return 0
}
run_tests r4_t5a.log 600 tests/test_tp_ipc.py
run_tests r4_t5b.log 900 tests/test_wide_deep.py tests/test_shuffle.py tests/test_dist_gpu.py tests/test_bench_launch.py tests/test_bert_tp.py
run_tests r4_t5c.log 600 tests/test_gemm.py tests/test_image_pipeline.py tests/test_parallel_gpu.py
for r in 1 2; do
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b5.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b5.json')); print('bench', round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2))"
done
bash tools/prof_run.sh bench_r4a 300 -- python3 bench.py --steps 200 --warmup 20
head -n 14 gpurun_out/bench_r4a_kernels.md
