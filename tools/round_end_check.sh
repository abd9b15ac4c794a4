timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/full_t.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
