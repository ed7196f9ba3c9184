# round 5: multi-rank bench flow rehearsal on one GPU (2 and 4 ranks sharing cuda:0, gloo) -- functional only
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for n in 2 4; do
  MIFX_SHARED_GPU=1 MIFX_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus $n --steps 10 --warmup 3 > gpurun_out/r5t_bench_$n.json 2> gpurun_out/r5t_bench_$n.err || { tail -30 gpurun_out/r5t_bench_$n.err; exit 1; }
  python -c "import json; r=json.loads([l for l in open('gpurun_out/r5t_bench_$n.json') if l.startswith('{')][-1]); print($n, 'ranks:', r['config'].get('dp_exchange'), 'bit_identical', r['config'].get('replicas_bit_identical'), 'ref', r['reference_batch'].get('dp_exchange'), r['reference_batch'].get('replicas_bit_identical'), 'validated', r['config'].get('validated_after_timed_region'))"
done
