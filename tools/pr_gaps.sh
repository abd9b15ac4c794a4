# Kernel durations and the idle gaps before each k_pr_pull_units launch in the PR bench
# (rocprofv3 kernel trace), per configuration:
#   gpurun -- bash tools/pr_gaps.sh name:ENV=V,ENV=V [name:...]
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "$@"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  env ${envs//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps_$name -o run -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/gaps_$name.json 2> gpurun_out/gaps_$name.err || exit 1
  python3 - "$name" "gpurun_out/gaps_$name/run_kernel_trace.csv" "gpurun_out/gaps_$name.json" <<'PY'
import csv, json, sys
rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
durs, gaps, prev = [], [], None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if "k_pr_pull" in r["Kernel_Name"]:
        durs.append((e - s) / 1e3)
        if prev is not None and s - prev < 100e3:
            gaps.append((s - prev) / 1e3)
    prev = e
d = json.load(open(sys.argv[3]))
print(f"{sys.argv[1]:>8}: pull {sum(durs)/len(durs):6.1f} us x {len(durs)}, gap before it {sum(gaps)/max(1,len(gaps)):5.1f} us; "
      f"bench {d['ms_per_step']:.4f} ms/step {d['value']/1e9:.1f} G", flush=True)
PY
done
