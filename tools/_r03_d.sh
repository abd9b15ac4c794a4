set -o pipefail
mkdir -p gpurun_out/d
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/d/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" > gpurun_out/d/rc.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/pr_ab.sh gpurun_out/d/ab SYN-7_5 2 "perm:GX_X=1" "noperm:GX_PR_LANEPERM=0" || exit 1
GX_PLAN_TIMES=1 GX_PR_VERBOSE=1 timeout -k 10 300 python bench.py --graph SYN-7_5 --no-secondary --cpu-seconds 0.1 --steps 3 --warmup 1 > gpurun_out/d/times_7_5.json 2> gpurun_out/d/times_7_5.err || exit 1
bash tools/pr_ab.sh gpurun_out/d/ab SYN-8_5 1 "perm:GX_X=1" "noperm:GX_PR_LANEPERM=0" || exit 1
GX_PLAN_TIMES=1 GX_PR_VERBOSE=1 timeout -k 10 300 python bench.py --graph SYN-8_5 --no-secondary --cpu-seconds 0.1 --steps 3 --warmup 1 > gpurun_out/d/times_8_5.json 2> gpurun_out/d/times_8_5.err || exit 1
bash tools/pr_probe.sh gpurun_out/d/probe SYN-7_5 "0 1 2 3 5 6" || exit 1
bash tools/pr_probe.sh gpurun_out/d/probe SYN-8_5 "0 1 2 3 5 6" || exit 1
