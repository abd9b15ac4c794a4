# PageRank launch time per entry as the graph shrinks under the Infinity Cache (256 MiB):
# index stream 4 B/entry (gpurun -- bash tools/pr_scale_probe.sh)
for sc in 18 19 20; do
  timeout -k 10 200 python bench.py --scale $sc --edgefactor 32 --seed 75 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prs.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/prs.json'));r=d['roofline'];print('scale $sc', round(d['value']/1e9,1), 'G edges/s', round(r['mean_launch_us'],1), 'us', round(r['frac'],3))"
done
