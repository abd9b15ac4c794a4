set -o pipefail
# WCC after a change: parity (small and full size), bench lines alternated with the scatter
# remap (GX_REMAP=scatter), and a rocprofv3 kernel-stats pass.  Usage: bash tools/wcc_check.sh [OUT]
O=${1:-gpurun_out/wcc_check}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "wcc or hub_first" > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fullsize.py tests/test_distributed.py -m gpu -k "wcc" > $O/t2.log 2>&1 || exit 1
for r in 1 2; do
  for v in gather scatter; do
    GX_REMAP=$v timeout -k 10 200 python bench.py --algorithm wcc --no-cpu-baseline > $O/wcc_${v}_$r.json 2> $O/wcc_${v}_$r.err || exit 1
    python3 -c "import json;d=json.loads(open('$O/wcc_${v}_$r.json').read().strip().splitlines()[-1]);print('$v $r', d['ms_per_step'], d['roofline']['frac'])" | tee -a $O/summary.txt
  done
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pw -o run -- python3 bench.py --algorithm wcc --no-cpu-baseline --steps 100 > $O/pw.json 2>&1
rc=$?
find $O -name "*kernel_trace.csv" -delete
exit $rc
