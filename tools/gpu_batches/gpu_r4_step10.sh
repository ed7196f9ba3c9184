# Round-4 GPU batch 10: fused FFN block (test + BERT A/B), BERT kernel table after the dX / FFN changes.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u tools/diag_resnet_graph.py > gpurun_out/resnet_graph_diag2_r4.jsonl 2> gpurun_out/resnet_graph_diag2_r4.err || { tail -5 gpurun_out/resnet_graph_diag2_r4.err; exit 1; }
cat gpurun_out/resnet_graph_diag2_r4.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm.py tests/test_bert_tp.py tests/test_tp_ipc.py -k "ffn or dx or transpose or bert or attention" > gpurun_out/r4_t10a.log 2>&1; rc=$?; tail -3 gpurun_out/r4_t10a.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for r in 1 2; do
for gb in 1 0; do
MIFX_HIP_GELU_BWD=$gb timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_ffn.json 2> gpurun_out/bert_ffn.err || { tail -5 gpurun_out/bert_ffn.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_ffn.json') if l.startswith('{')][-1]; print('gelu_bwd_fused', $gb, round(d['value'],1), round(d['ms_per_step'],3), d.get('calls_per_step_native_vs_fallback'))" | tee -a gpurun_out/bert_ffn_ab_r4.txt
done
done
timeout -k 10 400 python -u tools/torch_kernel_table.py --model bert --batch 32 --seq 128 --warmup 6 --active 3 > gpurun_out/bert_steady_r4b.md 2> gpurun_out/bert_steady_r4b.err || { tail -5 gpurun_out/bert_steady_r4b.err; exit 1; }
head -n 24 gpurun_out/bert_steady_r4b.md
