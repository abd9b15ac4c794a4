# SYN-cit CDLP x10: GX_CDLP_FIRST_GRID (the first pass grid cap in blocks)
set -o pipefail
mkdir -p gpurun_out/fg
for r in 1 2; do
for v in 2048 4096 8192 16384; do
  GX_CDLP_FIRST_GRID=$v timeout -k 10 180 python bench.py --algorithm cdlp --graph SYN-cit --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fg/cit_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fg/cit_$v.json'));print('SYN-cit first_grid=$v round $r', round(d['ms_per_step'],4), 'first', round(d['roofline']['kernels']['cdlp_first']['ms_per_run'],4))" | tee -a gpurun_out/fg/summary.txt
done
done
