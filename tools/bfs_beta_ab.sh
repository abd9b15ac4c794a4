set -o pipefail
# BFS beta 24 against 48 on undirected graphs, alternated.  Usage: bash tools/bfs_beta_ab.sh [OUT]
O=${1:-gpurun_out/bfs_beta_ab}; mkdir -p $O
for r in 1 2 3; do
  for G in SYN-g500-22 SYN-7_5; do
    for b in 24 48; do
      GX_BFS_BETA=$b timeout -k 10 200 python bench.py --algorithm bfs --graph $G --no-cpu-baseline --steps 300 --warmup 5 > $O/b.json 2> $O/b.err || exit 1
      python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$G beta $b run $r', d['ms_per_step'])" | tee -a $O/summary.txt
    done
  done
done
