# Round-4 GPU batch 20: one-launch step for one-workgroup batches (optimizer workgroups inside the fused launch):
# bit-identity tests, W&D suite, bench A/B at the reference batch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_wide_deep.py -k "one_launch" > gpurun_out/r4_t20a.log 2>&1 || { tail -30 gpurun_out/r4_t20a.log; exit 1; }
tail -1 gpurun_out/r4_t20a.log
true
true
for r in 1 2 3; do
for ol in 1 0; do
MIFX_WD_ONE_LAUNCH=$ol timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b20.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b20.json')); print('one_launch', $ol, round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2), d['config']['grad_check_max_rel_err_vs_fp32'])" | tee -a gpurun_out/wd_one_launch_ab_r4.txt
done
done
