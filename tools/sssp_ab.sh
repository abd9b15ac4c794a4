# SSSP bench over configuration switches (gpurun -- bash tools/sssp_ab.sh "ENV=V,ENV=V" ...)
G=${G:-SYN-8_5}
for cfg in "$@"; do
  env ${cfg//,/ } timeout -k 10 180 python bench.py --algorithm sssp --graph $G --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/sab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sab.json'));print('$G $cfg', round(d['ms_per_step'],3), d.get('parity_vs_oracle'))"
done
