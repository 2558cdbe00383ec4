O=gpurun_out/vh2; mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/with_cpu.json 2> $O/with_cpu.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/no_cpu.json 2> $O/no_cpu.err || exit 1
OMP_WAIT_POLICY=passive timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/with_cpu_passive.json 2> $O/with_cpu_passive.err || exit 1
nproc > $O/nproc.txt; cat /sys/fs/cgroup/cpu.max > $O/cpumax.txt 2>&1; cat /sys/fs/cgroup/cpu.stat >> $O/cpumax.txt 2>&1; echo ok
