# Round-4 GPU batch 21: LayerNorm-backward rows per wave (partial rows of the column reduction) on the BERT step.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bert_tp.py -k "layernorm or many_rows" > gpurun_out/r4_t21a.log 2>&1 || { tail -30 gpurun_out/r4_t21a.log; exit 1; }
tail -1 gpurun_out/r4_t21a.log
for r in 1 2; do
for rpw in 2 1 4; do
MIFX_BERT_LN_RPW=$rpw timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_rpw.json 2> gpurun_out/bert_rpw.err || { tail -5 gpurun_out/bert_rpw.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_rpw.json') if l.startswith('{')][-1]; print('ln_rpw', $rpw, round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_ln_rpw_ab_r4.txt
done
done
