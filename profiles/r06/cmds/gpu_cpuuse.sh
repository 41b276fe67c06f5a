# CPU consumed by a 16-thread queue_bench run (user / sys) and the cgroup's throttling counters around it
set -o pipefail
O=gpurun_out/cpuuse
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for mode in devupdate device; do
  { echo "== $mode"; cat /sys/fs/cgroup/cpu.stat; } >> $O/cpu.log 2>&1
  { time timeout -k 10 300 build/ctest/queue_bench 131072 16 $mode 64 ; } >> $O/cpu.log 2>&1 || exit 1
  cat /sys/fs/cgroup/cpu.stat >> $O/cpu.log 2>&1
  { time QB_CPU_QUEUE=0 timeout -k 10 300 build/ctest/queue_bench 131072 1 $mode 1024 ; } >> $O/cpu.log 2>&1 || exit 1
done
cat $O/cpu.log
