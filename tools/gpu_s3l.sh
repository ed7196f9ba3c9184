#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sweep_wd.py > gpurun_out/sweep_wd.log 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/sweep_wd.log; exit 1; }
grep batch gpurun_out/sweep_wd.log
