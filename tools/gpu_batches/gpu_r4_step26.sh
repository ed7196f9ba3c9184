# Round-4 GPU batch 26: embedding gradient written in the weight dtype (no fp32 image + cast): tests + BERT step.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bert_tp.py tests/test_tp_ipc.py > gpurun_out/r4_t26a.log 2>&1 || { tail -30 gpurun_out/r4_t26a.log; exit 1; }
tail -1 gpurun_out/r4_t26a.log
for r in 1 2 3; do
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_eg.json 2> gpurun_out/bert_eg.err || { tail -5 gpurun_out/bert_eg.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_eg.json') if l.startswith('{')][-1]; print('bert emb_bf16', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_emb_bf16_r4.txt
done
