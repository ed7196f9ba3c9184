# Round-4 GPU batch 8: record prefetch (tests + bench A/B), BERT dX on the NT kernel (tests + A/B), ResNet graph
# diagnosis, ResNet conv table with MIOpen through convolution_backward.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run_tests() {  # log, timeout, args...
  local log=$1 t=$2; shift 2
  timeout -k 10 "$t" python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests $log rc=$rc: stopping"; exit $rc; fi
  return 0
}
run_tests r4_t8a.log 600 tests/test_wide_deep.py tests/test_shuffle.py tests/test_gemm.py -k "prefetch or large_tile or shuffle or transpose or dx or nn"
for r in 1 2 3; do
for pf in 1 0; do
MIFX_WD_PREFETCH=$pf timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r4_b8.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r4_b8.json')); print('prefetch', $pf, round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2), d['config']['grad_check_max_rel_err_vs_fp32'])" | tee -a gpurun_out/wd_prefetch_ab_r4.txt
done
done
for r in 1 2; do
for dx in 1 0; do
MIFX_HIP_GEMM_DX=$dx timeout -k 10 400 python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 > gpurun_out/bert_dx.json 2> gpurun_out/bert_dx.err || { tail -5 gpurun_out/bert_dx.err; exit 1; }
python -c "import json; d=[json.loads(l) for l in open('gpurun_out/bert_dx.json') if l.startswith('{')][-1]; print('dx_nt', $dx, round(d['value'],1), round(d['ms_per_step'],3), d.get('calls_per_step_native_vs_fallback'))" | tee -a gpurun_out/bert_dx_ab_r4.txt
done
done
timeout -k 10 300 python -u tools/diag_resnet_graph.py > gpurun_out/resnet_graph_diag_r4.jsonl 2> gpurun_out/resnet_graph_diag_r4.err || { tail -5 gpurun_out/resnet_graph_diag_r4.err; exit 1; }
cat gpurun_out/resnet_graph_diag_r4.jsonl
timeout -k 10 600 python -u tools/bench_resnet_convs.py > gpurun_out/resnet_conv_routes_r4.jsonl 2> gpurun_out/resnet_conv_routes_r4.err || { tail -5 gpurun_out/resnet_conv_routes_r4.err; exit 1; }
tail -n 1 gpurun_out/resnet_conv_routes_r4.jsonl
