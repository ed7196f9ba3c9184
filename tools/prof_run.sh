#!/bin/bash
# usage: tools/prof_run.sh NAME TIMEOUT -- python3 ...   -> gpurun_out/NAME_kernels.md (raw .db removed)
set -o pipefail
name=$1; to=$2; shift 3
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 "$to" rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$name" -o "$name" -- "$@" > "gpurun_out/prof_$name.log" 2>&1 || { tail -20 "gpurun_out/prof_$name.log"; exit 1; }
db=$(find "gpurun_out/prof_$name" -name "*.db" | head -1)
python3 tools/prof_summary.py "$db" --out "gpurun_out/${name}_kernels.md" > /dev/null && rm -rf "gpurun_out/prof_$name"
echo "profile $name ok"
