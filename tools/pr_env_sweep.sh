#!/bin/bash
# PageRank launch time (bench.py roofline.mean_launch_us) over env settings, one bench run each.
# bash tools/pr_env_sweep.sh OUTDIR name:ENV=VAL,ENV=VAL ...   (BENCH_ARGS adds bench.py flags)
set -o pipefail
OUT=$1
shift
mkdir -p "$OUT"
for cfg in "$@"; do
    name=${cfg%%:*}
    envs=${cfg#*:}
    [ "$envs" = "$cfg" ] && envs=""
    env ${envs//,/ } timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-secondary --no-cpu-baseline $BENCH_ARGS \
        > "$OUT/$name.json" 2> "$OUT/$name.err" || exit 1
    tail -1 "$OUT/$name.json" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name [$envs]', round(r['mean_launch_us'],1), 'us per launch', round(d['ms_per_step'],3), 'ms per step', 'frac', round(r['frac'],3), flush=True)" | tee -a "$OUT/summary.txt"
done
