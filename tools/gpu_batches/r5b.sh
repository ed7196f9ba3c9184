set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm8.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r5b_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r5b_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/bench_gemm8.py --shapes bertdw > gpurun_out/r5b_dw.log 2>&1 || exit $?
cat gpurun_out/r5b_dw.log
for d in 1 0 1 0; do
  MIFX_DEFER_DW=$d timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/r5b_bert_defer$d.json 2> gpurun_out/r5b_bert_defer$d.err || exit $?
  python -c "import json,sys; r=json.loads(open('gpurun_out/r5b_bert_defer$d.json').read().strip().splitlines()[-1]); print('defer', $d, round(r['value'],1), 'seq/s', round(r['ms_per_step'],3), 'ms', r['loss'])"
done
