# BERT TP: row-parallel GEMM + peer-memory all-reduce overlapped in token chunks (side stream); TP tests (graph ==
# eager bit-identical at TP 2 / 4 with the overlap; overlapped == plain), TP=2 and TP=8 kernel tables with the
# stream-overlap summary (ranks sharing one GPU)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_tp_ipc.py tests/test_bert_tp.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/tpov_tests.log 2>&1 || { grep -E "Error|assert" gpurun_out/tpov_tests.log | head -20; tail -30 gpurun_out/tpov_tests.log; exit 1; }
tail -1 gpurun_out/tpov_tests.log
timeout -k 10 300 python -u tools/tp_kernel_table.py --tp 2 --layers 12 > gpurun_out/bert_tp2_overlap_r5.md 2> gpurun_out/tp2.err || { tail -20 gpurun_out/tp2.err; exit 1; }
grep -E "Streams|step:" gpurun_out/bert_tp2_overlap_r5.md
MIFX_TP_OVERLAP_CHUNKS=1 timeout -k 10 300 python -u tools/tp_kernel_table.py --tp 2 --layers 12 > gpurun_out/bert_tp2_nooverlap_r5.md 2> gpurun_out/tp2n.err || { tail -20 gpurun_out/tp2n.err; exit 1; }
grep -E "Streams|step:" gpurun_out/bert_tp2_nooverlap_r5.md
timeout -k 10 400 python -u tools/tp_kernel_table.py --tp 8 --layers 12 --steps 5 > gpurun_out/bert_tp8_overlap_r5.md 2> gpurun_out/tp8.err || { tail -20 gpurun_out/tp8.err; exit 1; }
grep -E "Streams|step:" gpurun_out/bert_tp8_overlap_r5.md
