#!/bin/bash
# Same-box A/B of the W&D bench between this tree and a built copy of another revision in ./ab_old (git archive +
# build: mkdir ab_old && git archive REV | tar -x -C ab_old && (cd ab_old && python -c "import __graft_entry__ as g; g.build()"));
# alternating processes; prints us/step at B=65536 and at the reference batch. Delete ab_old afterwards (it is
# git-ignored but travels with every gpurun call while it exists).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for run in 1 2 3; do
  for v in new old; do
    d=.; [ $v = old ] && d=ab_old
    (cd $d && timeout -k 10 200 python -u bench.py --steps ${1:-200} --warmup 20 > $OLDPWD/gpurun_out/abtree_$v$run.json 2>/dev/null) || exit 1
    python -c "import json;d=json.load(open('gpurun_out/abtree_$v$run.json'));print('$v',$run,round(d['ms_per_step']*1e3,2),round(d['reference_batch']['ms_per_step']*1e3,2))"
  done
done
