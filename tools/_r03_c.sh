set -o pipefail
mkdir -p gpurun_out/c
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/ -m gpu > gpurun_out/c/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc" > gpurun_out/c/rc.txt
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/pr_ab.sh gpurun_out/c/ab SYN-7_5 2 "new:GX_X=1" "noperm:GX_PR_LANEPERM=0" "nosfx:GX_PR_SUFFIX=0" || exit 1
bash tools/pr_ab.sh gpurun_out/c/ab SYN-8_5 1 "new:GX_X=1" "noperm:GX_PR_LANEPERM=0" "nosfx:GX_PR_SUFFIX=0" || exit 1
bash tools/pr_probe.sh gpurun_out/c/probe SYN-7_5 "0 1 2 3 5 6" || exit 1
