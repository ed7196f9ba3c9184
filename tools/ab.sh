#!/bin/bash
# Same-box A/B(/C...) of any benchmark command. Each round runs the command once per variant, alternating
# variants, every run a fresh process, so box-to-box and thermal drift cancel out of the comparison.
#
# usage: tools/ab.sh [-n ROUNDS] [-t SECONDS] [-o NAME] VARIANT... -- COMMAND [ARGS...]
#   VARIANT   LABEL[=VAR=VALUE[,VAR=VALUE...]]   environment for that variant (LABEL alone: unchanged env);
#             the pseudo-variable DIR=PATH runs the command from another built tree (e.g. ab_old, made with
#             mkdir ab_old && git archive REV | tar -x -C ab_old && (cd ab_old && python -c
#             "import __graft_entry__ as g; g.build()") -- delete it afterwards, it travels with every gpurun call)
#             a VALUE naming an existing relative path is made absolute (library overrides MIFX_LIB_<NAME>=...).
#   -n        rounds (default 2); -t per-run time limit in seconds (default 300); -o result name (default ab)
#
# Each run's stdout goes to gpurun_out/ab_<name>_<label><round>.log (stderr to .err), so a long run keeps
# writing under gpurun_out/; the last JSON line of stdout is appended to gpurun_out/ab_<name>.jsonl as
# {"variant": LABEL, "run": R, "result": {...}} and summarised on stdout (ms/step, reference-batch ms/step,
# loss and gradient check when the line carries them). Stops at the first failing run.
#
# examples (the round-3 A/Bs in profiles/*_ab_r3.txt):
#   tools/ab.sh -o bert_async dw1=MIFX_BERT_ASYNC_DW=1 dw0=MIFX_BERT_ASYNC_DW=0 -- python -u tools/bench_bert.py --steps 30
#   tools/ab.sh -n 3 -t 200 -o wd base prio=MIFX_LIB_WD_CHAIN=tools/bin/libwd_chain_prio.so,MIFX_LIB_WD_CHAIN64=tools/bin/libwd_chain64_prio.so -- python -u bench.py --steps 200 --warmup 20
#   tools/ab.sh -n 3 -t 200 -o tree new old=DIR=ab_old -- python -u bench.py --steps 200 --warmup 20
#   tools/ab.sh -t 400 -o bn new old=MIFX_LIB_BN_RELU=tools/bin/libbn_relu_old.so -- python -u -m mifx.trainer.resnet_trainer --steps 30
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
rounds=2; limit=300; name=ab
while getopts "n:t:o:" opt; do
  case $opt in n) rounds=$OPTARG ;; t) limit=$OPTARG ;; o) name=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
variants=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do variants+=("$1"); shift; done
[ "$1" = "--" ] && shift
if [ ${#variants[@]} -lt 1 ] || [ $# -lt 1 ]; then
  echo "usage: tools/ab.sh [-n ROUNDS] [-t SECONDS] [-o NAME] VARIANT... -- COMMAND [ARGS...]" >&2; exit 2
fi
root=$PWD
mkdir -p gpurun_out
for run in $(seq 1 "$rounds"); do
  for spec in "${variants[@]}"; do
    label=${spec%%=*}
    envs=(); dir=.
    if [ "$spec" != "$label" ]; then
      IFS=',' read -r -a assigns <<< "${spec#*=}"
      for a in "${assigns[@]}"; do
        key=${a%%=*}; val=${a#*=}
        if [ "$key" = DIR ]; then dir=$val; continue; fi
        [ -e "$val" ] && [ "${val#/}" = "$val" ] && val=$root/$val
        envs+=("$key=$val")
      done
    fi
    log=$root/gpurun_out/ab_${name}_${label}${run}
    echo "[ab] $label run $run: ${envs[*]} (cwd $dir)"
    (cd "$dir" && env "${envs[@]}" timeout -k 10 "$limit" "$@" > "$log.log" 2> "$log.err") \
      || { echo "[ab] $label run $run failed"; tail -20 "$log.err"; exit 1; }
    python - "$log.log" "$label" "$run" "$root/gpurun_out/ab_${name}.jsonl" <<'EOF' || exit 1
import json, sys
path, label, run, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
if not lines:
    sys.exit(f"[ab] {label} run {run}: no JSON line in {path}")
d = json.loads(lines[-1])
with open(out, "a") as f:
    f.write(json.dumps({"variant": label, "run": run, "result": d}) + "\n")
cols = [label, run]
if "ms_per_step" in d:
    cols.append(f"ms/step={d['ms_per_step']:.5g}")
rb = d.get("reference_batch") or {}
if "ms_per_step" in rb:
    cols.append(f"ref_ms/step={rb['ms_per_step']:.5g}")
if "loss" in d:
    cols.append(f"loss={d['loss']}")
g = (d.get("config") or {}).get("grad_check_max_rel_err_vs_fp32")
if g is not None:
    cols.append(f"grad_check={g:.3g}")
print(*cols)
EOF
  done
done
