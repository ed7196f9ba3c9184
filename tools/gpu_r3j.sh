#!/bin/bash
# PATE ensemble kernel trace (250 teachers only)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pate_prof3 -o pate -- python3 tools/bench_pate.py --steps 12 --teachers 250 --no-sequential > gpurun_out/pate_prof3.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/pate_prof3.log; exit 1; }
echo done
