# round 5: BERT FFN dH GEMM (GELU-backward epilogue) on the pipelined kernel vs the one-barrier kernel (A/B)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MIFX_GELU_BWD_G8=1 timeout -k 10 300 python -u -m pytest tests/test_bert_tp.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ffn or gelu" > gpurun_out/r5q_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r5q_tests.log; [ $rc -eq 0 ] || [ $rc -eq 5 ] || { tail -30 gpurun_out/r5q_tests.log; exit 1; }
for v in 0 1 0 1; do
  MIFX_GELU_BWD_G8=$v timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 10 > gpurun_out/r5q_bert_$v.json 2> gpurun_out/r5q_bert_$v.err || { tail -20 gpurun_out/r5q_bert_$v.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5q_bert_$v.json') if l.startswith('{')][-1]); print('gelu_bwd_g8', $v, round(r['value'],1), round(r['ms_per_step'],3), 'ms', 'loss', r.get('loss'))"
done
