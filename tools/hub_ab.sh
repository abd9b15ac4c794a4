# Warm-call A/B of the hub-first copy (GX_HUB=0 never, 1 from the second call) for BFS, WCC
# and SSSP on their default graphs: gpurun -- bash tools/hub_ab.sh
mkdir -p gpurun_out
for a in bfs wcc sssp; do
  for h in 0 1; do
    GX_HUB=$h timeout -k 10 300 python bench.py --algorithm $a --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/hub_${a}_$h.json 2> gpurun_out/hub_${a}_$h.err || exit 1
    python -c "import json;d=json.load(open('gpurun_out/hub_${a}_$h.json'));print('$a GX_HUB=$h', round(d['ms_per_step'],3), 'ms; first call', round(d['first_call_ms'],1), 'ms')"
  done
done
