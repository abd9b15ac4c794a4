set -o pipefail
# SSSP bucket-width scale (GX_SSSP_DSCALE) on the undirected config graphs.
# Usage: bash tools/sssp_dscale_sweep.sh [OUT]
O=${1:-gpurun_out/sssp_dscale}; mkdir -p $O
for G in SYN-8_5 SYN-g500-22 SYN-7_5; do
  for sc in 3 1.5 2 1 3; do
    GX_SSSP_DSCALE=$sc timeout -k 10 200 python bench.py --algorithm sssp --graph $G --no-cpu-baseline --steps 60 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$G dscale $sc', d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
