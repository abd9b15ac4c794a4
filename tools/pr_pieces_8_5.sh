# Per-piece PageRank launch on SYN-8_5 at N = 1 with P pieces (P = 8: the per-rank SpMV of an
# 8-GPU run; 16: 8 GPUs x 2 pipelined pieces).  gpurun -- bash tools/pr_pieces_8_5.sh
mkdir -p gpurun_out/pieces
for P in 1 8 16; do
  GX_PR_PIECES=$P timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --graph SYN-8_5 --steps 10 --warmup 2 --no-cpu-baseline \
      > gpurun_out/pieces/p85_$P.json 2> gpurun_out/pieces/p85_$P.err || exit 1
  tail -1 gpurun_out/pieces/p85_$P.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SYN-8_5 P=$P', round(d['roofline']['mean_launch_us'],1), 'us per piece launch', round(d['ms_per_step'],3), 'ms per PR', d['config'].get('exchanged_doubles_per_n'), flush=True)"
done
