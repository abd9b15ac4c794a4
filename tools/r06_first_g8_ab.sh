# SYN-cit CDLP x10: GX_CDLP_FIRST_G8 (rows up to this many entries merged by 8-lane groups; 0: off)
set -o pipefail
mkdir -p gpurun_out/f8
for r in 1 2; do
for v in 0 12 16 24; do
  GX_CDLP_FIRST_G8=$v timeout -k 10 180 python bench.py --algorithm cdlp --graph SYN-cit --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/f8/cit_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/f8/cit_$v.json'));print('SYN-cit first_g8=$v round $r', round(d['ms_per_step'],4), 'first', round(d['roofline']['kernels']['cdlp_first']['ms_per_run'],4))" | tee -a gpurun_out/f8/summary.txt
done
done
