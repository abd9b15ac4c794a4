set -o pipefail
mkdir -p gpurun_out/r5n
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k cdlp --timeout 150 --timeout-method thread > gpurun_out/r5n/cdlp_parity.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_fullsize.py -x -q -k cdlp --timeout 280 --timeout-method thread > gpurun_out/r5n/cdlp_full.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --algorithm cdlp --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r5n/cdlp.json 2> gpurun_out/r5n/cdlp.err || exit 1
timeout -k 10 850 bash tools/r04_unit_sweep.sh gpurun_out/r5n/sweep > gpurun_out/r5n/sweep.log 2>&1 || exit 1
for q in 0 1; do GX_PR_QUEUE=$q GX_PR_PIECES=8 timeout -k 10 200 python3 bench.py --partitioned --steps 30 --no-cpu-baseline --no-secondary > gpurun_out/r5n/pieces_q$q.json 2> gpurun_out/r5n/pieces_q$q.err || exit 1; done
