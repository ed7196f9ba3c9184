#!/bin/bash
# Round-6 rehearsal part B: smoke, the 1-GPU bench with its default flags, configs 4 / 5, rocprof kernel tables of the
# headline step and the BERT step (summaries only; trace databases deleted on the box).
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_rehearsal.log 2>&1 || { tail -20 gpurun_out/smoke_rehearsal.log; exit 1; }
tail -1 gpurun_out/smoke_rehearsal.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_rehearsal.json 2> gpurun_out/bench_rehearsal.err || { tail -20 gpurun_out/bench_rehearsal.err; exit 1; }
cut -c1-300 gpurun_out/bench_rehearsal.json
timeout -k 10 300 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_rehearsal.json 2> gpurun_out/bert_rehearsal.err || { tail -20 gpurun_out/bert_rehearsal.err; exit 1; }
grep '^{' gpurun_out/bert_rehearsal.json | tail -1 | cut -c1-300
timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_rehearsal.json 2> gpurun_out/resnet_rehearsal.err || { tail -20 gpurun_out/resnet_rehearsal.err; exit 1; }
grep '^{' gpurun_out/resnet_rehearsal.json | tail -1 | cut -c1-300
MIFX_DP_FORCE=1 timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/resnet_dp_forced_rehearsal.json 2> gpurun_out/resnet_dp_forced_rehearsal.err || { tail -20 gpurun_out/resnet_dp_forced_rehearsal.err; exit 1; }
grep '^{' gpurun_out/resnet_dp_forced_rehearsal.json | tail -1 | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_wd -o run -- python -u bench.py --steps 50 --warmup 10 > gpurun_out/r6/prof_wd.log 2>&1 || { tail -20 gpurun_out/r6/prof_wd.log; exit 1; }
python tools/prof_summary.py gpurun_out/r6/prof_wd/run_results.db --title "W&D headline step (bench.py, B=65536, 50 timed steps), rocprofv3 kernel trace, round 6" --out gpurun_out/r6/bench_r6_kernels.md > /dev/null
python tools/timeline.py gpurun_out/r6/prof_wd/run_results.db --last 12 --match wdc_fused,wd_reduce_res,wd_res_opt > gpurun_out/r6/bench_r6_timeline.txt 2>&1 || true
rm -rf gpurun_out/r6/prof_wd
head -12 gpurun_out/r6/bench_r6_kernels.md
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_bert -o run -- python -u -m mifx.trainer.bert_trainer --steps 10 --warmup 5 > gpurun_out/r6/prof_bert.log 2>&1 || { tail -20 gpurun_out/r6/prof_bert.log; exit 1; }
python tools/step_window.py gpurun_out/r6/prof_bert/run_results.db --marker adamw --top 40 > gpurun_out/r6/bert_steady_r6.md
rm -rf gpurun_out/r6/prof_bert
head -8 gpurun_out/r6/bert_steady_r6.md
echo done
