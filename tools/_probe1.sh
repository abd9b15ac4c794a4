set -o pipefail
mkdir -p gpurun_out/p1
{ nproc; python3 -c "import os;print('affinity',len(os.sched_getaffinity(0)),'cpu_count',os.cpu_count())"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /proc/self/cgroup; env | grep -E 'OMP|MAX_JOBS|THREADS' ; free -g; } > gpurun_out/p1/env.txt 2>&1
timeout -k 10 300 python3 bench.py --graph SYN-8_5 --steps 10 --warmup 2 --cpu-seconds 5 > gpurun_out/p1/bench85.json 2> gpurun_out/p1/bench85.err
