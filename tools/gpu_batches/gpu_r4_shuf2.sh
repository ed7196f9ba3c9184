# A/B of the record-shuffle granularity: groups of 4 records (default build) vs per-record (tools/bin *_g1 builds,
# -DMIFX_SHUFFLE_GLOG2=0, loaded through the MIFX_LIB_* overrides) vs no shuffle; alternating processes, 2 rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/wd_shuffle_ab_r4.txt
echo "# bench.py --steps 20 --warmup 5 (B=65536 T=256 kernel, B=40 T=64 kernel); columns: variant run us/step(B=65536) us/step(B=40) grad_check" > $out
for r in 1 2 3; do
for v in g4 g1 none; do
  case $v in
    g4) env_="" ; seed=24301 ;;
    g1) env_="MIFX_LIB_WD_CHAIN256=tools/bin/libwd_chain256_g1.so MIFX_LIB_WD_CHAIN64=tools/bin/libwd_chain64_g1.so" ; seed=24301 ;;
    none) env_="" ; seed=0 ;;
  esac
  env $env_ timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --shuffle-seed $seed > gpurun_out/shab.json 2>gpurun_out/shab.err || { tail -5 gpurun_out/shab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/shab.json')); print('$v', $r, round(d['ms_per_step']*1e3,2), round(d['reference_batch']['ms_per_step']*1e3,2), d['config']['grad_check_max_rel_err_vs_fp32'])" >> $out
done; done
cat $out
