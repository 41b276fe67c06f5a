# host-cell queue throughput after the idle-close change (device queue's CPU route, CPU executor), 2 repetitions
set -o pipefail
O=gpurun_out/qhost2
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for rep in 1 2; do
  for C in 32768 131072 1048576; do
    for T in 1 8 16; do
      timeout -k 10 120 build/ctest/queue_bench $C $T >> $O/route.log 2>&1 || exit 1
    done
    QB_CPU_QUEUE=1 timeout -k 10 120 build/ctest/queue_bench $C 16 >> $O/cpuq.log 2>&1 || exit 1
    timeout -k 10 120 build/ctest/queue_bench $C 16 update 64 >> $O/route_update.log 2>&1 || exit 1
  done
done
grep -h '^{' $O/*.log
