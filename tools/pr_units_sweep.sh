#!/bin/bash
# PageRank bench over plan configurations (split-block size, unit size, block shape).
# Run on the GPU box:
#   gpurun -- bash tools/pr_units_sweep.sh GRAPH name:ENV=VAL,ENV=VAL [name:...]
# e.g. bash tools/pr_units_sweep.sh SYN-7_5 u1:GX_PR_BLOCK_UNITS=1 u8:GX_PR_BLOCK_UNITS=8
mkdir -p gpurun_out
G=${1:-SYN-7_5}
shift
for cfg in "$@"; do
    name=${cfg%%:*}
    envs=${cfg#*:}
    env ${envs//,/ } timeout -k 10 240 python bench.py --graph "$G" --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/sweep_${G}_$name.json 2> gpurun_out/sweep_${G}_$name.err || exit $?
    python - "$name" "$envs" "gpurun_out/sweep_${G}_$name.json" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[3]).read())
r = d["roofline"]
print(f"{sys.argv[1]:>10} {sys.argv[2]:60s} {d['value']/1e9:7.1f} G edges/s  {d['ms_per_step']:.3f} ms/PR  "
      f"launch {r['mean_launch_us']:.1f} us  frac {r['frac']:.3f}", flush=True)
EOF
done
