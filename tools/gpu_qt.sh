# queue batch phase timing (diagnostic build in qt_tmp/, not committed)
set -o pipefail
mkdir -p gpurun_out/qt
make -s -C tests/c queue_bench || exit 1
for m in device devupdate; do
  for C in 131072 1048576; do
    LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench $C 16 $m 64 >> gpurun_out/qt/qt.log 2>&1 || exit 1
  done
done
LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 1 device 256 >> gpurun_out/qt/qt.log 2>&1 || exit 1
cat gpurun_out/qt/qt.log
