set -o pipefail
mkdir -p gpurun_out/fd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fd/tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/fd/n1.json 2> gpurun_out/fd/n1.err || exit 1
GX_PR_PIECES=8 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fd/p8.json 2> gpurun_out/fd/p8.err || exit 1
echo ok
