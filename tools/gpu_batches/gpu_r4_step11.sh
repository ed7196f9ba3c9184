# Round-4 GPU batch 11: transpose cache (test + BERT bench), ResNet graph test, W&D bench check.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm.py tests/test_parallel_gpu.py tests/test_tp_ipc.py -k "transpose or ffn or dx or resnet or bert" > gpurun_out/r4_t11a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t11a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2 3; do
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_tc.json 2> gpurun_out/bert_tc.err || { tail -5 gpurun_out/bert_tc.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_tc.json') if l.startswith('{')][-1]; print('bert tcache', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_tcache_r4.txt
done
grep "^{" gpurun_out/bert_tc.json > gpurun_out/bert_r4c.json
