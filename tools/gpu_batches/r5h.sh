# round 5: data-parallel bucket exchange on peer-memory kernels captured with the backward (one graph per step)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_parallel_gpu.py tests/test_tp_ipc.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r5h_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r5h_tests.log | tail -20; [ $rc -eq 0 ] || { tail -60 gpurun_out/r5h_tests.log; exit $rc; }
run() {  # label, env...
  local lab=$1; shift
  env "$@" timeout -k 10 400 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/r5h_$lab.json 2> gpurun_out/r5h_$lab.err || { tail -20 gpurun_out/r5h_$lab.err; return 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5h_$lab.json') if l.startswith('{')][-1]); print('$lab', round(r['value'],1), round(r['ms_per_step'],3), 'ms', r.get('dp_exchange'), 'graphs/step', r.get('graphs_per_step'))"
}
for i in 1 2; do
  run nodp_defer0 MIFX_DEFER_DW=0 && run dp1_ipc MIFX_DP_FORCE=1 MIFX_DP_EXCHANGE=ipc && run dp1_rccl MIFX_DP_FORCE=1 MIFX_DP_EXCHANGE=rccl && run nodp_default MIFX_DEFER_DW=1 || exit 1
done
