# queue device-update batches: launch sub-phases and the worker's thread CPU time (diagnostic build qt_tmp/)
set -o pipefail
O=gpurun_out/qt9
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for T in 1 4 16; do
  for rep in 1 2; do
    echo "== threads $T" >> $O/qt.log
    LD_LIBRARY_PATH=qt_tmp timeout -k 10 300 build/ctest/queue_bench 131072 $T devupdate $((1024 / T)) >> $O/qt.log 2>&1 || exit 1
  done
done
cat $O/qt.log
