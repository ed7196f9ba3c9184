# Round-4 GPU batch 24: non-temporal state accesses in the flat AdamW (BERT step A/B) + AdamW tests.
set -o pipefail
mkdir -p gpurun_out
MIFX_ADAMW_NT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "adamw" > gpurun_out/r4_t24a.log 2>&1; rc=$?; tail -1 gpurun_out/r4_t24a.log
if [ $rc -ne 0 ] && [ $rc -ne 5 ]; then tail -30 gpurun_out/r4_t24a.log; exit 1; fi
for r in 1 2; do
for nt in 1 0; do
MIFX_ADAMW_NT=$nt timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_nt.json 2> gpurun_out/bert_nt.err || { tail -5 gpurun_out/bert_nt.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_nt.json') if l.startswith('{')][-1]; print('adamw_nt', $nt, round(d['value'],1), round(d['ms_per_step'],3))" | tee -a gpurun_out/bert_adamw_nt_ab_r4.txt
done
done
