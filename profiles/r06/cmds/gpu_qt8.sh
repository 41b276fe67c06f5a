# queue batch phase timing: 2 vs 8 pointer-table scratch slots per context (diagnostic builds qt_tmp/, qt8/)
set -o pipefail
O=gpurun_out/qt8
mkdir -p $O
make -s -C tests/c queue_bench || exit 1
for rep in 1 2; do
  for lib in qt_tmp qt8; do
    for mode in devupdate device; do
      echo "== $lib $mode" >> $O/qt.log
      LD_LIBRARY_PATH=$lib timeout -k 10 300 build/ctest/queue_bench 131072 16 $mode 64 >> $O/qt.log 2>&1 || exit 1
    done
  done
done
cat $O/qt.log
