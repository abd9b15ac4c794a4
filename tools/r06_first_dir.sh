# Directed CDLP first-iteration shortcut: parity tests, SYN-cit A/B (GX_CDLP_FIRST_SORTED)
# gpurun -- bash tools/r06_first_dir.sh
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k cdlp \
  > gpurun_out/fd/tests.log 2>&1 || { tail -30 gpurun_out/fd/tests.log; exit 1; }
tail -3 gpurun_out/fd/tests.log
for r in 1 2; do
for v in 1 0; do
  GX_CDLP_FIRST_SORTED=$v timeout -k 10 180 python bench.py --algorithm cdlp --graph SYN-cit --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/fd/cit_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/fd/cit_$v.json'));print('SYN-cit first_sorted=$v round $r', round(d['ms_per_step'],4), d['roofline']['kernels'])" | tee -a gpurun_out/fd/summary.txt
done
done
