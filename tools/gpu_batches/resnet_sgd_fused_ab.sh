# ResNet-50 captured SGD: torch foreach passes vs the fused multi-tensor kernel (csrc/sgd.hip, MIFX_SGD_FUSED):
# SGD / trainer GPU tests, step A/B, kernel stats of the fused step
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_sgd_fused.py tests/test_parallel_gpu.py tests/test_image_pipeline.py -m gpu -x -q -k "sgd or resnet" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/sgd_tests.log 2>&1 || { tail -30 gpurun_out/sgd_tests.log; exit 1; }
tail -1 gpurun_out/sgd_tests.log; grep -c PASSED gpurun_out/sgd_tests.log || true
for f in 0 1 0 1; do
  MIFX_SGD_FUSED=$f timeout -k 10 300 python -u -m mifx.trainer.resnet_trainer --steps 20 --warmup 5 > gpurun_out/sgd_resnet.json 2> gpurun_out/sgd_resnet.err || { tail -20 gpurun_out/sgd_resnet.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/sgd_resnet.json') if l.startswith('{')][-1]); print('fused', $f, r.get('sgd'), round(r['value'],1), round(r['ms_per_step'],3), 'ms')"
done
R=$PWD
for f in 0 1; do
  (cd /tmp && export TMPDIR=/tmp && PYTHONPATH=$R MIFX_SGD_FUSED=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/sgdprof_$f -o run -- python3 -m mifx.trainer.resnet_trainer --steps 6 --warmup 4 > $R/gpurun_out/sgd_prof_$f.log 2>&1) || { tail -20 gpurun_out/sgd_prof_$f.log; exit 1; }
  python3 - $f <<'PY'
import csv, glob, sys
f = glob.glob(f"/tmp/sgdprof_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for row in csv.DictReader(open(f)):
    n = row["Name"]
    if "sgd_chunks" in n or "multi_tensor_apply" in n:
        print("fused", sys.argv[1], n[:70], "calls", row["Calls"], "total_us", round(float(row["TotalDurationNs"]) / 1e3, 1), "avg_us", round(float(row["AverageNs"]) / 1e3, 1))
PY
done
