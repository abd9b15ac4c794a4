set -o pipefail
mkdir -p ${OUT:-gpurun_out/dist}
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -m gpu -x -v --timeout 120 --timeout-method thread > ${OUT:-gpurun_out/dist}/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > ${OUT:-gpurun_out/dist}/n1.json 2> ${OUT:-gpurun_out/dist}/n1.err || exit 1
for P in 1 2 8; do
GX_PR_PIECES=$P timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > ${OUT:-gpurun_out/dist}/d$P.json 2> ${OUT:-gpurun_out/dist}/d$P.err || exit 1
GX_PR_GRAPH=0 GX_PR_PIECES=$P timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 20 --warmup 3 --no-cpu-baseline > ${OUT:-gpurun_out/dist}/ng$P.json 2> ${OUT:-gpurun_out/dist}/ng$P.err || exit 1
done
