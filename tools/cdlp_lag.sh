# CDLP bench with the host's flag lag 1 vs 2 and sparse-only off/on (gpurun -- bash tools/cdlp_lag.sh)
for gr in SYN-7_5 SYN-cit; do
  for cfg in "GX_CDLP_LAG=1" "GX_CDLP_LAG=2" "GX_CDLP_SPARSE_ONLY=0" "GX_CDLP_SPARSE=0"; do
    env $cfg timeout -k 10 120 python bench.py --algorithm cdlp --graph $gr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/lag.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/lag.json'));print('$gr $cfg', round(d['ms_per_step'],3), round(d['wall_ms_per_call_incl_d2h'],3))"
  done
done
