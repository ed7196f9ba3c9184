#!/bin/bash
# Multi-rank bench.py flow rehearsed on ONE GPU (functional only: ranks share cuda:0, timings mean nothing):
# torchrun with N ranks, xGMI exchange setup + self-test + post-run validation, then the reference batch.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 MIFX_SHARED_GPU=1 MIFX_DIST_BACKEND=gloo
mkdir -p gpurun_out
N=${1:-2}
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29611 bench.py --gpus $N --steps 20 --warmup 5 --ref-steps 200 > gpurun_out/bench_shared_$N.json \
  2> gpurun_out/bench_shared_$N.err
rc=$?
cat gpurun_out/bench_shared_$N.json | cut -c1-400
grep -E "xGMI|fall|fail|Error" gpurun_out/bench_shared_$N.err | head -5
exit $rc
