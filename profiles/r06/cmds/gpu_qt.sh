# queue batch phase timing (diagnostic build in qt_tmp/): placement queries per request 4 vs 2
set -o pipefail
mkdir -p gpurun_out/qt3
make -s -C tests/c queue_bench || exit 1
for rep in 1 2 3; do
  LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 16 devupdate 64 >> gpurun_out/qt3/qt.log 2>&1 || exit 1
  QB_ONE_ALLOC=1 LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 16 devupdate 64 >> gpurun_out/qt3/qt.log 2>&1 || exit 1
done
cat gpurun_out/qt3/qt.log
