set -o pipefail
# Result remap of the hub-first copy, scatter (default) against gather (GX_REMAP=gather):
# parity of the hub-copy tests under gather, then bench lines alternated.  Usage: bash tools/remap_ab.sh [OUT]
O=${1:-gpurun_out/remap_ab}; mkdir -p $O
GX_REMAP=gather timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hub_first or bfs or sssp or wcc" > $O/t.log 2>&1 || exit 1
for r in 1 2; do
 for v in scatter gather; do
  for A in "bfs SYN-g500-22" "wcc SYN-g500-22" "sssp SYN-8_5"; do
   set -- $A
   GX_REMAP=$v timeout -k 10 200 python bench.py --algorithm $1 --graph $2 --no-cpu-baseline --steps 200 --warmup 5 > $O/b_${v}_$1_$r.json 2> $O/b_${v}_$1_$r.err || exit 1
   python3 -c "import json;d=json.loads(open('$O/b_${v}_$1_$r.json').read().strip().splitlines()[-1]);print('$v $1 $2 $r', d['ms_per_step'])" | tee -a $O/summary.txt
  done
 done
done
