#!/bin/bash
# PageRank launch time over (edgefactor, unit entries T, block entries B) on R-MAT scale 20
# (bench.py --edgefactor); one line per run.  bash tools/pr_ts_sweep.sh "32:T1,T2 24:T1" "B1 B2"
mkdir -p gpurun_out/ts
for spec in $1; do
  ef=${spec%%:*}; ts=${spec#*:}
  for t in ${ts//,/ }; do
    for b in $2; do
      GX_PR_UNIT_NNZ=$t GX_PR_BLOCK_NNZ=$b GX_PR_LONG_NNZ=$t timeout -k 10 200 python3 bench.py --edgefactor $ef \
          --no-cpu-baseline --steps 20 > gpurun_out/ts/ef${ef}_${t}_${b}.json 2>/dev/null || exit 1
      tail -1 gpurun_out/ts/ef${ef}_${t}_${b}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('ef $ef T $t B $b', round(r['mean_launch_us'],1), 'us', round(r['frac'],3), flush=True)"
    done
  done
done
