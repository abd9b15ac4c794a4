# BFS bench over configuration switches (gpurun -- bash tools/bfs_ab.sh "ENV=V,ENV=V" ...)
for G in SYN-g500-22 SYN-cit; do
for cfg in "$@"; do
  env ${cfg//,/ } timeout -k 10 180 python bench.py --algorithm bfs --graph $G --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bab.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bab.json'));print('$G $cfg', round(d['ms_per_step'],3), round(d['value']/1e9,1))"
done
done
