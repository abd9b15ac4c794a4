#!/bin/bash
# Per-piece PageRank launch time at N = 1 with P pieces (= the per-rank SpMV of a P-GPU run)
# over plan settings.  bash tools/pr_piece_sweep.sh P name:ENV=VAL,ENV=VAL ...
mkdir -p gpurun_out/pieces
P=$1
shift
for cfg in "$@"; do
    name=${cfg%%:*}
    envs=${cfg#*:}
    env ${envs//,/ } GX_PR_PIECES=$P timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline \
        > gpurun_out/pieces/p${P}_$name.json 2> gpurun_out/pieces/p${P}_$name.err || exit 1
    tail -1 gpurun_out/pieces/p${P}_$name.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('P=$P $name $envs', round(d['roofline']['mean_launch_us'],1), 'us per piece launch', round(d['ms_per_step'],3), 'ms per PR', flush=True)"
done
