#!/bin/bash
# Round 3: first-round prefetch (default build) against a build without it (tools/pf0), and the
# launch simulation with fitted unit costs for SYN-7_5 (GX_PR_SIM=1).
set -o pipefail
OUT=${1:-gpurun_out/pf}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py -k "pagerank or narrow or PR" > "$OUT/pytest_pr.log" 2>&1 || { tail -30 "$OUT/pytest_pr.log"; exit 1; }
tail -1 "$OUT/pytest_pr.log"
bash tools/pr_ab.sh "$OUT" SYN-7_5 2 "pf1:GX_PR_SIM=0" "pf0:GX_LIB=tools/pf0/libgx.so" \
    "sim:GX_PR_SIM=1,GX_PR_SIM_RATE=5500,GX_PR_SIM_ROW=1700,GX_PR_SIM_FIXED=3600" || exit 1
bash tools/pr_ab.sh "$OUT" SYN-8_5 1 "pf1:GX_PR_SIM=0" "pf0:GX_LIB=tools/pf0/libgx.so" || exit 1
echo pf-ok
