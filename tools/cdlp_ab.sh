# CDLP bench over configuration switches (gpurun -- bash tools/cdlp_ab.sh "ENV=V,ENV=V" ...)
for gr in SYN-7_5 SYN-cit; do
  for cfg in "$@"; do
    env ${cfg//,/ } timeout -k 10 120 python bench.py --algorithm cdlp --graph $gr --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$gr $cfg', round(d['ms_per_step'],3), round(d['first_call_ms'],1))"
  done
done
