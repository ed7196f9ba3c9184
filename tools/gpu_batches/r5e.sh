# round 5: fused 1x1 ResNet path after routing the 1x1 backward to MIOpen and the two-level BN tile finalize
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_conv1x1.py tests/test_gemm8.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5e_tests.log; [ $rc -eq 0 ] || { tail -40 gpurun_out/r5e_tests.log; exit $rc; }
for v in "1 1" "0 0" "1 1" "0 0"; do
  set -- $v
  MIFX_RESNET_FUSED_1X1=$1 MIFX_DEFER_DW=$2 timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5e_resnet_$1$2.json 2> gpurun_out/r5e_resnet_$1$2.err || { tail -20 gpurun_out/r5e_resnet_$1$2.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5e_resnet_$1$2.json') if l.startswith('{')][-1]); print('fused', $1, 'defer', $2, round(r['value'],1), r.get('unit'), round(r.get('ms_per_step',0),3), 'ms')"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r5e_prof -o r5e -- python3 -m mifx.trainer.resnet_trainer --steps 10 --warmup 3 > gpurun_out/r5e_prof.log 2>&1 || { tail -20 gpurun_out/r5e_prof.log; exit 1; }
f=$(find gpurun_out/r5e_prof -name "*kernel_stats.csv" | head -1); head -45 "$f" | cut -d, -f1-4 | cut -c1-160
