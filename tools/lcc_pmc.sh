# PMC passes over LCC on SYN-cit (gpurun -- bash tools/lcc_pmc.sh)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc_lcc1 -o run -- python bench.py --algorithm lcc --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_lcc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d gpurun_out/pmc_lcc2 -o run -- python bench.py --algorithm lcc --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_lcc2.log 2>&1 || exit 1
