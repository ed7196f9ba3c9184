# Round-4 GPU batch 15: kernel-argument placement (HIP_FORCE_DEV_KERNARG) on the W&D step and prologue stamps.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
for kv in unset 1 0; do
if [ $kv = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$kv; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b15.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b15.json')); print('dev_kernarg', '$kv', round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2))" | tee -a gpurun_out/wd_kernarg_ab_r4.txt
done
done
unset HIP_FORCE_DEV_KERNARG
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python -u tools/stamps_wdc.py --quick > gpurun_out/wdc_stamps_devka.txt 2>&1 || exit 1
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 300 python -u tools/stamps_wdc.py --quick > gpurun_out/wdc_stamps_hostka.txt 2>&1 || exit 1
grep -E "==|prologue" gpurun_out/wdc_stamps_devka.txt gpurun_out/wdc_stamps_hostka.txt
