# Round-4 GPU batch 25: column reductions (one-pass few-row sums; 8-column reduce blocks): tests + BERT step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bert_tp.py tests/test_gemm.py -k "col_sum or gelu or ffn or layernorm or bert" > gpurun_out/r4_t25a.log 2>&1 || { tail -30 gpurun_out/r4_t25a.log; exit 1; }
tail -1 gpurun_out/r4_t25a.log
for r in 1 2 3; do
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_cs.json 2> gpurun_out/bert_cs.err || { tail -5 gpurun_out/bert_cs.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_cs.json') if l.startswith('{')][-1]; print('bert redcols32', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_redcols32_r4.txt
done
