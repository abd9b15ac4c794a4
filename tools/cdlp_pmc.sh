# PMC counters of the CDLP kernels (gpurun -- bash tools/cdlp_pmc.sh GRAPH)
G=${1:-SYN-7_5}; ALG=${2:-cdlp}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_cdlp -o run -- python bench.py --algorithm $ALG --graph $G --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_cdlp.log 2>&1
