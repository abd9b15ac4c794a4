#!/bin/bash
# Multi-GPU (vertex-range) algorithm paths through RCCL on the GPUs of one box.
# Usage (repo root): bash tools/bench_partitioned.sh OUTDIR NGPUS [alg ...]
set -o pipefail
OUT=${1:-gpurun_out/part}
NG=${2:-1}
shift 2
ALGS=${@:-bfs wcc cdlp lcc sssp}
mkdir -p "$OUT"
for a in $ALGS; do
    timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$NG" --master-addr 127.0.0.1 \
        --master-port $((29500 + RANDOM % 1000)) bench.py --algorithm $a --gpus "$NG" --partitioned --steps 3 --warmup 1 \
        > "$OUT/$a.json" 2> "$OUT/$a.err"
    rc=$?
    echo "$a rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$a.err"; exit $rc; }
    python3 -c "
import json
d=json.loads(open('$OUT/$a.json').read().strip().splitlines()[-1])
print(f\"{d['config']['workload']:34s} N={d['n_gpus']} {d['value']/1e9:8.2f} G{d['unit']}  {d['ms_per_step']:.2f} ms  parity {d['parity_vs_oracle']}\")
"
done
