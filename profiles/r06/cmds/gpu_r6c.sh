# queue on device cells: update per-request cost vs encode, one vs two allocations
set -o pipefail
mkdir -p gpurun_out/r6c
make -s -C tests/c queue_bench || exit 1
for C in 131072 1048576; do
  timeout -k 10 300 build/ctest/queue_bench $C 16 device 64 >> gpurun_out/r6c/qb.log 2>&1 || exit 1
  timeout -k 10 300 build/ctest/queue_bench $C 16 devupdate 64 >> gpurun_out/r6c/qb.log 2>&1 || exit 1
  QB_ONE_ALLOC=1 timeout -k 10 300 build/ctest/queue_bench $C 16 devupdate 64 >> gpurun_out/r6c/qb.log 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6c/prof -o qb -- build/ctest/queue_bench 131072 16 devupdate 64 > gpurun_out/r6c/qb_prof.log 2>&1 || exit 1
echo ALLDONE
