# host-cell updates computed on the CPU by the queue (CPU executor / device queue's host route) after the
# accumulate-in-place change; encodes for reference
set -o pipefail
O=gpurun_out/cpuupd
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for C in 131072 1048576; do
  for T in 1 16; do
    timeout -k 10 120 build/ctest/queue_bench $C $T update 64 >> $O/route_update.log 2>&1 || exit 1
    QB_CPU_QUEUE=1 timeout -k 10 120 build/ctest/queue_bench $C $T update 64 >> $O/cpuq_update.log 2>&1 || exit 1
    QB_CPU_QUEUE=1 timeout -k 10 120 build/ctest/queue_bench $C $T >> $O/cpuq_encode.log 2>&1 || exit 1
  done
done
cat $O/*.log | grep '^{'
