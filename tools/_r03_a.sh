set -o pipefail
mkdir -p gpurun_out/a
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/a/gpu_tests.log 2>&1
rc=$?
echo "gpu tests rc=$rc" > gpurun_out/a/rc.txt
# a fault, abort, segfault or time limit ends the call; assertion failures (rc 1) do not
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/a/bench.json 2> gpurun_out/a/bench.err || exit 1
bash tools/pr_probe.sh gpurun_out/a/probe SYN-7_5 || exit 1
bash tools/pr_probe.sh gpurun_out/a/probe SYN-8_5 "0 2 3 1" || exit 1
