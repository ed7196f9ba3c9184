# Round-4 GPU batch 16: LayerNorm forward with gamma/beta hoisted, chunked deterministic embedding backward:
# numerics tests, BERT step, steady-state kernel table.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bert_tp.py -k "layernorm or ln_gelu or fused_add or bias_dropout or embedding or bitwise or tp_dropout" > gpurun_out/r4_t16a.log 2>&1 || { tail -20 gpurun_out/r4_t16a.log; exit 1; }
tail -1 gpurun_out/r4_t16a.log
for r in 1 2 3; do
timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_ln.json 2> gpurun_out/bert_ln.err || { tail -5 gpurun_out/bert_ln.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_ln.json') if l.startswith('{')][-1]; print('bert ln', round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_ln_r4.txt
done
timeout -k 10 400 python -u tools/torch_kernel_table.py --model bert --batch 32 --warmup 6 --active 3 > gpurun_out/bert_steady_r4d.md 2> gpurun_out/bert_table.err || { tail -5 gpurun_out/bert_table.err; exit 1; }
grep -E "add_ln|GPU time" gpurun_out/bert_steady_r4d.md
