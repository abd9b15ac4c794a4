#!/bin/bash
# rocprofv3 kernel-trace summaries of the per-algorithm bench lines (one MI355X).
# Usage (repo root, GPU box): bash tools/profile_algorithms.sh OUTDIR [alg ...]
# Writes OUTDIR/<alg>/..._kernel_stats.csv and copies each summary to
# OUTDIR/r01_<alg>_kernel_stats.csv (commit those under profiles/).
set -o pipefail
OUT=${1:-gpurun_out/algprof}
shift
ALGS=${@:-bfs wcc cdlp lcc sssp}
mkdir -p "$OUT"
export TMPDIR=/tmp
for a in $ALGS; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$a" -o "$a" -- \
        python3 bench.py --algorithm $a --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/$a.log" 2>&1
    rc=$?
    echo "$a rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/$a.log"; exit $rc; }
    f=$(find "$OUT/$a" -name "*kernel_stats.csv" | head -1)
    [ -n "$f" ] && cp "$f" "$OUT/r01_${a}_kernel_stats.csv"
done
