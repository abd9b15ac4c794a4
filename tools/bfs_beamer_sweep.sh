set -o pipefail
# Beamer's direction-switch thresholds (GX_BFS_ALPHA / GX_BFS_BETA) swept on the device-driven
# BFS.  Usage: bash tools/bfs_beamer_sweep.sh [OUT]
O=${1:-gpurun_out/bfs_beamer}; mkdir -p $O
for G in SYN-g500-22 SYN-cit; do
  for ab in "14 24" "8 24" "24 24" "14 12" "14 48" "8 12" "24 48" "14 24"; do
    set -- $ab
    GX_BFS_ALPHA=$1 GX_BFS_BETA=$2 timeout -k 10 200 python bench.py --algorithm bfs --graph $G --no-cpu-baseline --steps 300 --warmup 5 > $O/b_${G}_$1_$2.json 2> $O/b.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/b_${G}_$1_$2.json').read().strip().splitlines()[-1]);print('$G alpha $1 beta $2', d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
