#!/bin/bash
# Round-end GPU suite (run on the MI355X box from the repo root): pytest -m gpu, smoke, the default bench line.
set -o pipefail
mkdir -p gpurun_out/fa
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > gpurun_out/fa/full_t.log 2>&1; rc=$?; tail -3 gpurun_out/fa/full_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fa/smoke.log 2>&1 || exit 1
tail -2 gpurun_out/fa/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/fa/bench_default.json 2> gpurun_out/fa/bench_default.err || exit 1
tail -c 600 gpurun_out/fa/bench_default.json
