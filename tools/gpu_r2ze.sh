#!/bin/bash
# Round 2: rehearsal of the driver's multi-rank bench flow on ONE GPU (gloo ranks sharing cuda:0; timings meaningless)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 MIFX_DIST_BACKEND=gloo MIFX_SHARED_GPU=1
for n in 2 4; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29550 + n)) bench.py --gpus $n --steps 20 --warmup 5 --data-per-gpu 4194304 > gpurun_out/bench_shared_$n.json 2> gpurun_out/bench_shared_$n.err || { tail -30 gpurun_out/bench_shared_$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_shared_$n.json').read().strip().splitlines()[-1]); print($n, d['n_gpus'], d['config']['dp_exchange'], d['config']['replicas_bit_identical'], d['reference_batch']['dp_exchange'], round(d['value']/1e6,1), 'M ex/s (shared GPU)')"
  grep -i "fall\|unavailable\|error" gpurun_out/bench_shared_$n.err | head -5
done
