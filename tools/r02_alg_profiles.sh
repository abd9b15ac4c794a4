# Round-2 bench lines (with the CPU baseline and parity) and rocprofv3 kernel summaries of the
# same commands for BFS, WCC and SSSP on their default graphs:
#   gpurun -- bash tools/r02_alg_profiles.sh
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r02alg
for a in bfs wcc sssp; do
  timeout -k 10 300 python bench.py --algorithm $a --steps 5 --warmup 2 > gpurun_out/r02alg/bench_$a.json 2> gpurun_out/r02alg/bench_$a.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02alg/prof_$a -o run -- \
    python bench.py --algorithm $a --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r02alg/prof_$a.json 2> gpurun_out/r02alg/prof_$a.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02alg/bench_$a.json'));print('$a', round(d['ms_per_step'],3), 'ms', round(d['value']/1e9,1), d['unit'], d['parity_vs_oracle'], 'cpu', round(d['cpu_baseline']['value']/1e9,3))"
done
