#!/bin/bash
# LCC dense-core A/B on SYN-cit (config 5): GX_LCC_CORE = the core's largest size (0: the hash
# kernels only).  One bench line per setting on OUT, parity against the oracle on each; prints
# device ms.  Usage (repo root, MI355X box): bash tools/lcc_core_ab.sh OUT "0 2048 4096 8192"
set -o pipefail
OUT=${1:-gpurun_out/lcc_core}
mkdir -p "$OUT"
for k in ${2:-0 2048 4096 8192}; do
  GX_LCC_CORE=$k timeout -k 10 300 python bench.py --algorithm lcc --steps 10 --warmup 2 \
      > "$OUT/lcc_core_$k.json" 2> "$OUT/lcc_core_$k.err" || exit 1
  python3 -c "
import json; d=json.loads(open('$OUT/lcc_core_$k.json').read().strip().splitlines()[-1])
print('GX_LCC_CORE=$k', 'device %.3f ms' % d['ms_per_step'], 'first call %.1f ms' % d['first_call_ms'],
      'parity', d['parity_vs_oracle'], 'kernels', {k: round(v['ms_per_run'], 3) for k, v in d['roofline']['kernels'].items()})" \
      | tee -a "$OUT/summary.txt"
done
