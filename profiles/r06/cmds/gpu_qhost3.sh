# host-cell queue after "close a CPU batch early only when it is the queue's only work": throughput + latency
set -o pipefail
O=gpurun_out/qhost3
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
for C in 32768 131072 1048576; do
  QB_LATENCY=1 timeout -k 10 120 build/ctest/queue_bench $C 1 >> $O/latency.log 2>&1 || exit 1
  QB_LATENCY=1 timeout -k 10 120 build/ctest/queue_bench $C 1 update 64 >> $O/latency.log 2>&1 || exit 1
done
grep -h '^{' $O/*.log
