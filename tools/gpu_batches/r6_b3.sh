#!/bin/bash
# Round 6, batch 3:
#  1. sequence parallelism: IPC reduce-scatter / all-gather exactness, BERT SP step (ranks sharing the GPU); BERT
#     fused-op tests (dropout / LayerNorm mask offset)
#  2. BERT-base A/B: short attention kernels with 160-B LDS rows (new) vs 144-B rows (tools/bin/libattention_ld72.so)
#  3. W&D headline with the residue-class reduction as the default
set -o pipefail
mkdir -p gpurun_out/r6
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_tp_ipc.py::test_ipc_reduce_scatter_all_gather_exact" \
  "tests/test_tp_ipc.py::test_bert_sequence_parallel_captured_bit_identical_and_tracks_tp" \
  tests/test_bert_tp.py -m gpu \
  > gpurun_out/r6/b3_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" gpurun_out/r6/b3_tests.log | tail -30; tail -5 gpurun_out/r6/b3_tests.log; exit 1; }
tail -2 gpurun_out/r6/b3_tests.log
bash tools/ab.sh -n 2 -t 300 -o bert_ld ld80 ld72=MIFX_LIB_ATTENTION=tools/bin/libattention_ld72.so -- python -u -m mifx.trainer.bert_trainer --steps 30 --warmup 5 || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > gpurun_out/r6/bench_res.json 2> gpurun_out/r6/bench_res.err || { tail -20 gpurun_out/r6/bench_res.err; exit 1; }
grep '^{' gpurun_out/r6/bench_res.json | tail -1 | cut -c1-400
echo done
