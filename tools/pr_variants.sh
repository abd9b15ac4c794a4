#!/bin/bash
# Tuning session for k_pr_pull on the GPU box: plan-time variants + PMC counters.
# Usage (from the repo root, on the MI355X box): bash tools/pr_variants.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/variants}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # name, env..., -- bench args
    local name=$1; shift
    env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --warmup 2 > "$OUT/$name.json" 2> "$OUT/$name.err"
    local rc=$?
    python - "$OUT/$name.json" "$name" <<'EOF'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{sys.argv[2]:24s} launch {r['mean_launch_us']:8.1f} us  frac {r['frac']:.3f}  value {d['value']/1e9:7.2f} GE/s")
except Exception as e:
    print(sys.argv[2], "failed", e)
EOF
    return $rc
}
run stride1_nb2048 X=1 || exit 1
run stride1_nb1024 GX_PR_STREAM_NNZ=1024 || exit 1
run stride1_nb4096 GX_PR_STREAM_NNZ=4096 || exit 1
run int4 GX_PR_INT4=1 || exit 1
run hub GX_PR_KERNEL=hub || exit 1
rocprofv3 -L > "$OUT/counters.txt" 2>&1
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    tag=$(echo $set | cut -d' ' -f1)
    timeout -k 10 240 rocprofv3 --pmc $set --kernel-include-regex k_pr_pull --output-format csv -d "$OUT/pmc_$tag" -o pmc \
        -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/pmc_$tag.log" 2>&1
    echo "pmc $tag rc=$?"
done
