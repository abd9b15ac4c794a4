set -o pipefail
# SSSP knobs re-swept after the round-5 changes (bucket width scale, dense-opening divisor, pull
# fraction), alternated with the defaults.  Usage: bash tools/sssp_knob_sweep.sh [OUT]
O=${1:-gpurun_out/sssp_knobs}; mkdir -p $O
for r in 1 2; do
  for e in ${KNOBS:-"" "GX_SSSP_DSCALE=2" "GX_SSSP_DSCALE=2.5" "GX_SSSP_DSCALE=4" "GX_SSSP_DENSE=8" "GX_SSSP_DENSE=32" "GX_SSSP_PULL_FRAC=4" "GX_SSSP_PULL_FRAC=16"}; do
    env $e timeout -k 10 200 python bench.py --algorithm sssp --no-cpu-baseline --steps 60 --warmup 3 > $O/b.json 2> $O/b.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('run $r [${e:-default}]', d['ms_per_step'])" | tee -a $O/summary.txt
  done
done
