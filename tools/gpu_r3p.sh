#!/bin/bash
# headline bench kernel table (end of round 2): rocprofv3 kernel stats of bench.py at its default flags
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bench_prof -o bench -- python3 bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || { tail -5 gpurun_out/bench_prof.err; exit 1; }
tail -1 gpurun_out/bench_prof.json
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > gpurun_out/bench_200.json 2> gpurun_out/bench_200.err || { tail -5 gpurun_out/bench_200.err; exit 1; }
tail -1 gpurun_out/bench_200.json
