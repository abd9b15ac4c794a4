timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "cdlp or CDLP" > gpurun_out/cdlp_t.log 2>&1 || exit 1
for gr in SYN-7_5 SYN-cit; do timeout -k 10 120 python bench.py --algorithm cdlp --graph $gr --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/cdlp_$gr.json 2> gpurun_out/cdlp_$gr.err || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for gr in SYN-7_5 SYN-cit; do timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_$gr -o run -- python bench.py --algorithm cdlp --graph $gr --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/tr_$gr.log 2>&1 || exit 1; done
