#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stamps_wd.py > gpurun_out/stamps_8w.txt 2>&1 || { echo "stamps failed"; tail -20 gpurun_out/stamps_8w.txt; exit 1; }
cat gpurun_out/stamps_8w.txt
