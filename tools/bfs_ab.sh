set -o pipefail
# BFS A/B: parity tests, then the bench with the round-5 level changes (new) and without (old). Usage: bash tools/bfs_ab.sh [OUT]
O=${1:-gpurun_out/bfs_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "bfs or hub_first" > $O/t1.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fullsize.py -m gpu -k "bfs" > $O/t2.log 2>&1 || exit 1
for r in 1 2; do
 for v in new old; do
  for G in SYN-g500-22 SYN-cit; do
   if [ $v = old ]; then E="${OLD_ENV:-GX_BFS_NEXTBITS=0 GX_BFS_GRID=8192}"; else E=""; fi
   env $E timeout -k 10 200 python bench.py --algorithm bfs --graph $G --no-cpu-baseline --steps 200 --warmup 5 > $O/b_${v}_${G}_$r.json 2> $O/b_${v}_${G}_$r.err || exit 1
   python3 -c "import json;d=json.loads(open('$O/b_${v}_${G}_$r.json').read().strip().splitlines()[-1]);print('$v $G $r', d['ms_per_step'], d['roofline']['frac'])" | tee -a $O/summary.txt
  done
 done
done
