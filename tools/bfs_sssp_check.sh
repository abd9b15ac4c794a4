set -o pipefail
# BFS / SSSP after a change to their step drivers: parity (small, split, full size, multi), two
# bench lines each, and a rocprofv3 kernel-stats pass of each.  Usage: bash tools/bfs_sssp_check.sh [OUT]
O=${1:-gpurun_out/bfs_sssp_check}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_sssp_split.py -m gpu -k "hub_first or bfs or sssp or split" > $O/t1.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fullsize.py tests/test_distributed.py -m gpu -k "bfs or sssp" > $O/t2.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --algorithm bfs --no-cpu-baseline > $O/bfs_$r.json 2> $O/bfs_$r.err || exit 1
  timeout -k 10 300 python bench.py --algorithm sssp --no-cpu-baseline > $O/sssp_$r.json 2> $O/sssp_$r.err || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pb -o run -- python3 bench.py --algorithm bfs --no-cpu-baseline --steps 100 > $O/pb.json 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ps -o run -- python3 bench.py --algorithm sssp --no-cpu-baseline --steps 50 > $O/ps.json 2>&1
rc=$?
find $O -name "*kernel_trace.csv" -delete
exit $rc
