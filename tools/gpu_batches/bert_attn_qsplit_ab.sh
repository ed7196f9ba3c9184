# BERT-base attention forward split over queries (MIFX_ATTN_QSPLIT 1 / 2 / 4 workgroups per (batch, head)): tests, step A/B
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for q in 2 4; do
  MIFX_ATTN_QSPLIT=$q timeout -k 10 300 python -u -m pytest tests/test_bert_tp.py -m gpu -x -q -k "attention or attn" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/qsplit_tests_$q.log 2>&1 || { tail -30 gpurun_out/qsplit_tests_$q.log; exit 1; }
  tail -1 gpurun_out/qsplit_tests_$q.log
done
for q in 1 2 4 1 2 4; do
  MIFX_ATTN_QSPLIT=$q timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/qsplit_bert_$q.json 2> gpurun_out/qsplit_bert_$q.err || { tail -20 gpurun_out/qsplit_bert_$q.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/qsplit_bert_$q.json') if l.startswith('{')][-1]); print('qsplit', $q, round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
