#!/bin/bash
# One parameterised GPU-session runner (replaces the one-off tools/gpu_r*.sh scripts of earlier rounds).
#
#   tools/gpu_run.sh STEP [STEP ...]
#
# Every STEP runs under its own `timeout -k 10`, writes its log under gpurun_out/, and the session stops at the
# first failing step (no GPU work after a fault, abort, or time limit). Steps:
#   tests[:<pytest selection>]   pytest -m gpu (default: the whole tests/ dir), e.g. tests:tests/test_gconv.py
#   smoke                        __graft_entry__.smoke()
#   bench[:<extra args>]         bench.py --gpus 1 --steps 20 --warmup 5 [extra args, '+' separated]
#   pipeline[:<extra args>]      tools/pipeline_bench.py --device cuda [extra args, '+' separated]
#   py:<script>[:<args>]         python -u <script> <args '+' separated>
#   prof:<name>:<script>[:<args>] rocprofv3 --kernel-trace --stats -d gpurun_out/<name> -- python3 <script> <args>
# TIMEOUT=<seconds> overrides the per-step limit (default 600).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LIMIT=${TIMEOUT:-600}
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=""
  [[ "$step" == *:* ]] && rest=${step#*:}
  log=gpurun_out/step${n}_${kind}.log
  echo "[gpu_run] step $n: $step" >&2
  case "$kind" in
    tests)
      sel=${rest:-tests}
      timeout -k 10 "$LIMIT" python -u -m pytest ${sel//+/ } -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > "$log" 2>&1
      rc=$?
      grep -E "PASSED|FAILED|ERROR|^E " "$log" | tail -40
      tail -1 "$log" ;;
    smoke)
      timeout -k 10 "$LIMIT" python -u -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1
      rc=$?
      tail -3 "$log" ;;
    bench)
      timeout -k 10 "$LIMIT" python -u bench.py --gpus 1 --steps 20 --warmup 5 ${rest//+/ } > "$log" 2> "$log.err"
      rc=$?
      cat "$log"; [ $rc -eq 0 ] || tail -20 "$log.err" ;;
    pipeline)
      timeout -k 10 "$LIMIT" python -u tools/pipeline_bench.py --device cuda ${rest//+/ } > "$log" 2> "$log.err"
      rc=$?
      cat "$log"; [ $rc -eq 0 ] || tail -20 "$log.err" ;;
    py)
      script=${rest%%:*}
      args=""
      [[ "$rest" == *:* ]] && args=${rest#*:}
      timeout -k 10 "$LIMIT" python -u "$script" ${args//+/ } > "$log" 2> "$log.err"
      rc=$?
      tail -30 "$log"; [ $rc -eq 0 ] || tail -20 "$log.err" ;;
    prof)
      name=${rest%%:*}
      r2=${rest#*:}
      script=${r2%%:*}
      args=""
      [[ "$r2" == *:* ]] && args=${r2#*:}
      (cd /tmp && true)
      export TMPDIR=/tmp
      timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats -d "gpurun_out/$name" -o "$name" -- \
        python3 "$script" ${args//+/ } > "$log" 2> "$log.err"
      rc=$?
      tail -5 "$log"; [ $rc -eq 0 ] || tail -20 "$log.err" ;;
    *)
      echo "unknown step kind: $kind" >&2
      exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "[gpu_run] step $n ($step) failed with exit $rc: stopping" >&2
    exit $rc
  fi
done
