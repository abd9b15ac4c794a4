# kernel trace of SYN-cit CDLP with the directed first-iteration shortcut
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/fdp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fdp/prof -o run -- python bench.py --algorithm cdlp --graph SYN-cit --steps 3 --warmup 1 --no-cpu-baseline --pmc-traffic committed > gpurun_out/fdp/b.json 2> gpurun_out/fdp/b.err || { tail -5 gpurun_out/fdp/b.err; exit 1; }
f=$(find gpurun_out/fdp/prof -name '*kernel_stats.csv' | head -1)
grep -E "first|gather|Name" "$f"
