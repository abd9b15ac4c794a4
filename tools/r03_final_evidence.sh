#!/bin/bash
# Round 3 evidence: PageRank unit times + rocprofv3 trace/PMC (both graphs), SSSP PMC, the full
# GPU suite, smoke() and the default bench line.
set -o pipefail
mkdir -p gpurun_out
bash tools/r03_pr_evidence.sh gpurun_out/ev || exit 1
bash tools/alg_pmc.sh gpurun_out/alg_sssp sssp > gpurun_out/alg_sssp.log 2>&1 || { tail -20 gpurun_out/alg_sssp.log; exit 1; }
bash tools/round_end_check.sh || exit 1
tail -1 gpurun_out/full_t.log
cat gpurun_out/smoke.log
echo final-evidence-ok
