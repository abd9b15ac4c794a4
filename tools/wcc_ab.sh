# WCC bench over configuration switches (gpurun -- bash tools/wcc_ab.sh "ENV=V,ENV=V" ...)
for G in SYN-g500-22 SYN-cit; do
for cfg in "$@"; do
  env ${cfg//,/ } timeout -k 10 180 python bench.py --algorithm wcc --graph $G --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/wab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/wab.json'));print('$G $cfg', round(d['ms_per_step'],3), d['roofline']['kernels'])"
done
done
