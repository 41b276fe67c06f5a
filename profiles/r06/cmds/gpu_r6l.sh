# queue after the fetch-kernel table upload, the placement cache and unlocked launches: verified runs, then the
# device-cell encode and update matrices (3 repetitions each)
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
QB_VERIFY=1 timeout -k 10 120 build/ctest/queue_bench 131072 16 devupdate 16 > $O/verify.log 2>&1 || exit 1
QB_VERIFY=1 timeout -k 10 120 build/ctest/queue_bench 131072 16 device 16 >> $O/verify.log 2>&1 || exit 1
cat $O/verify.log
for C in 131072 1048576; do
  for T in 1 4 16; do
    for rep in 1 2 3; do
      timeout -k 10 300 build/ctest/queue_bench $C $T devupdate $((1024 / T)) >> $O/devupdate.log 2>&1 || exit 1
    done
  done
done
for C in 32768 131072 1048576; do
  for T in 1 4 16; do
    for rep in 1 2 3; do
      timeout -k 10 300 build/ctest/queue_bench $C $T device $((1024 / T)) >> $O/device.log 2>&1 || exit 1
    done
  done
done
echo ALLDONE
