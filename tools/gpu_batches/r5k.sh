# round 5: per-shape 3x3 convolution routing data; DP exchange diagnostic
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u tools/bench_conv3x3.py > gpurun_out/r5k_conv3x3.jsonl 2> gpurun_out/r5k_conv3x3.err || { tail -20 gpurun_out/r5k_conv3x3.err; exit 1; }
cat gpurun_out/r5k_conv3x3.jsonl
timeout -k 10 600 python -u tools/dp_exchange_diag.py > gpurun_out/r5k_dpdiag.json 2> gpurun_out/r5k_dpdiag.err || { tail -30 gpurun_out/r5k_dpdiag.err; exit 1; }
cat gpurun_out/r5k_dpdiag.json
