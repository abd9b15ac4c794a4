#!/bin/bash
# Round 3: unit records carry their block's fields; GX_PR_NARROW_MIN A/B; PR parity.
set -o pipefail
OUT=${1:-gpurun_out/nmin}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -1 "$OUT/pytest_pr.log"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "m0:GX_PR_NARROW_MIN=0" "m16k:GX_PR_NARROW_MIN=16384" "m64k:GX_PR_NARROW_MIN=65536" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-8_5 1 "m0:GX_PR_NARROW_MIN=0" "m64k:GX_PR_NARROW_MIN=65536" || exit 1
echo nmin-ok
