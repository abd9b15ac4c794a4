set -o pipefail
mkdir -p gpurun_out/final
bash tools/profile_round.sh gpurun_out/final/prof > gpurun_out/final/prof.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit 1
echo final-ok
